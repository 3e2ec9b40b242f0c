# One GPU session's evidence: gpu tests, default bench (CPU baselines), rocprof kernel stats, PMC passes
# (FETCH/WRITE for cfg3 and cfg2, SQ instruction mix and waits for the rollout kernel), cfg5/cfg2 lines.
# Usage (from the repo root on the GPU box): bash tools/gpu_round.sh <tag> [skip_tests]
set -e
tag=${1:-rXX}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
if [ "${2:-}" != "skip_tests" ]; then
  timeout -k 10 800 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
fi
timeout -k 10 400 python3 -u bench.py > $out/cfg3_bench.json 2> $out/cfg3_bench.err
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o p \
  -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu --no-exact > $out/cfg3_rocprof_bench.json 2> $out/rocprof.err
for cfgname in cfg3 cfg2; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex "k_roll_|k_walk_search" --output-format csv \
      -d $out/pmc_$cfgname/$c -o p \
      -- python3 -u bench.py --config $cfgname --steps 1 --warmup 0 --no-cpu --no-exact --horizon-ms 500 \
      > $out/pmc_${cfgname}_$c.log 2>&1
  done
done
g_waits="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
g_mix="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_BRANCH"
i=0
for g in "$g_waits" "$g_mix"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $g --kernel-include-regex "k_roll_|k_walk_search" --output-format csv \
    -d $out/pmc_sq/g$i -o p \
    -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --no-exact --horizon-ms 500 > $out/pmc_sq_g$i.log 2>&1
done
timeout -k 10 300 python3 -u bench.py --config cfg5 > $out/cfg5_bench.json 2> $out/cfg5_bench.err
timeout -k 10 240 python3 -u bench.py --config cfg2 > $out/cfg2_bench.json 2> $out/cfg2_bench.err
echo done
