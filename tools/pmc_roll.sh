# rocprofv3 PMC passes (one counter group per run) for the rollout kernels of a short cfg3 bench run.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcr
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_roll_" --output-format csv -d gpurun_out/pmcr/$c -o p \
    -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --horizon-ms 500 > gpurun_out/pmcr/$c.log 2>&1
done
