# One GPU session's evidence: gpu tests, default bench (CPU baseline), rocprof kernel stats, PMC passes, cfg5/cfg2 lines.
# Usage (from the repo root on the GPU box): bash tools/gpu_round.sh <tag>
set -e
tag=${1:-rXX}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/gpu_tests.log 2>&1
timeout -k 10 300 python3 -u bench.py > $out/cfg3_bench.json 2> $out/cfg3_bench.err
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o p \
  -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu > $out/cfg3_rocprof_bench.json 2> $out/rocprof.err
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex "k_roll_" --output-format csv -d $out/pmc/$c -o p \
    -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu --horizon-ms 500 > $out/pmc_$c.log 2>&1
done
timeout -k 10 300 python3 -u bench.py --config cfg5 > $out/cfg5_bench.json 2> $out/cfg5_bench.err
timeout -k 10 180 python3 -u bench.py --config cfg2 --no-cpu > $out/cfg2_bench.json 2> $out/cfg2_bench.err
echo done
