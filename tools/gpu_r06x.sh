# Round 6: (1) the appended-node search with optimize samples on their own lanes (option nn_lane_order, build var_lo):
# the lag-2 parity tests and cfg3 lines; (2) with that search off the overflow split's path, the split's total work is
# what it costs: the overflow budgets raised (fewer records, longer single-wave walks) and the walk grid at 2560.
# Usage (repo root on the GPU box): bash tools/gpu_r06x.sh <tag>
set -e
tag=${1:-r06x}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CLRRT_LIB=$GRAFT_REPO_ROOT/cl-rrt_amd/var_lo/libclrrt.so timeout -k 10 600 python -u -m pytest tests/test_full_size_parity.py \
  tests/test_gpu_parity.py tests/test_dist_gpu.py -m gpu -v -s --timeout 300 --timeout-method thread \
  -k "walk or brute or bench_size or late_query or bench_settings or deferred or pipelined or sharded" > $out/gpu_tests_lo.log 2>&1
grep -E "passed|failed" $out/gpu_tests_lo.log | tail -n 1
run() {
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact "$@" > $out/cfg3_bench_$name.json \
    2> $out/cfg3_bench_$name.err
  echo "$name $(cut -c1-90 $out/cfg3_bench_$name.json)"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['round_split'])" $out/cfg3_bench_$name.json
}
name=default; run
export CLRRT_LIB=$GRAFT_REPO_ROOT/cl-rrt_amd/var_lo/libclrrt.so
name=lo; run
name=lo_off; run --opt nn_lane_order=0
unset CLRRT_LIB
name=bk8k; run --opt nn_walk_budget_keys=8192
name=bt6k; run --opt nn_walk_budget_tiles=6144
name=ww2560; run --opt nn_walk_waves=2560
export CLRRT_LIB=$GRAFT_REPO_ROOT/cl-rrt_amd/var_lo/libclrrt.so
name=lo2; run
echo done
