# rocprofv3 PMC passes (one counter group per run) for the persistent rollout kernel on a short cfg3 bench
# run: instruction issue / wait cycles and instruction-cache behaviour.
# Usage (GPU box, repo root): bash tools/pmc_icache.sh <out_dir>
set -e
out=${1:-gpurun_out/pmci}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p $out
i=0
for g in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_IFETCH SQ_INSTS_LDS" \
         "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $g --kernel-include-regex "k_roll_run" --output-format csv -d $out/g$i -o p \
    -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --no-exact --horizon-ms 400 > $out/g$i.log 2>&1
done
