# Round 5 profiling session of the current build: rocprof kernel stats of the default bench command, PMC passes
# (FETCH/WRITE for cfg3 and cfg2, SQ wave state of the walk, SQ lane utilisation of the rollout kernel), recorded with
# the sources' fingerprint (tools/summarize_pmc.py "_src") so bench.py quotes passes of this build.
# Usage (repo root on the GPU box): bash tools/gpu_r05b.sh <tag> <commit>
set -e
tag=${1:-r05b}
build=${2:-unknown}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o p \
  -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu --no-exact --no-sync > $out/cfg3_rocprof_bench.json 2> $out/rocprof.err
for cfgname in cfg3 cfg2; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex "k_roll_run|k_walk_search" --output-format csv \
      -d $out/pmc_$cfgname/$c -o p \
      -- python3 -u bench.py --config $cfgname --steps 1 --warmup 0 --no-cpu --no-exact --no-sync --horizon-ms 500 \
      > $out/pmc_${cfgname}_$c.log 2>&1
  done
  python3 tools/summarize_pmc.py --build $build $out/pmc_$cfgname/FETCH_SIZE/p_counter_collection.csv > $out/${cfgname}_pmc_fetch.json
  python3 tools/summarize_pmc.py --build $build $out/pmc_$cfgname/WRITE_SIZE/p_counter_collection.csv > $out/${cfgname}_pmc_write.json
  rm -f $out/pmc_$cfgname/*/p_counter_collection.csv
done
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
  --kernel-include-regex "k_walk_search" --output-format csv -d $out/walk_sq -o p -- python3 -u bench.py --steps 1 --warmup 0 \
  --no-cpu --no-exact --no-sync --horizon-ms 1000 > $out/walk_sq.log 2>&1
python3 tools/summarize_pmc.py --build $build $out/walk_sq/p_counter_collection.csv > $out/cfg3_walk_sq.json
rm -f $out/walk_sq/p_counter_collection.csv
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU \
  --kernel-include-regex "k_roll_run" --output-format csv -d $out/roll_sq -o p -- python3 -u bench.py --steps 1 --warmup 0 \
  --no-cpu --no-exact --no-sync --horizon-ms 500 > $out/roll_sq.log 2>&1
python3 tools/summarize_pmc.py --build $build $out/roll_sq/p_counter_collection.csv > $out/cfg3_roll_sq.json
rm -f $out/roll_sq/p_counter_collection.csv
echo done
