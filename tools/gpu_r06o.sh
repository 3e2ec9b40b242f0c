# Round 6: the split appended-node search on the merge stream (no stream of its own): the GPU suite, then cfg3 bench
# lines of the committed build (var_head) and the working build with the split off / on.
# Usage (repo root on the GPU box): bash tools/gpu_r06o.sh <tag>
set -e
tag=${1:-r06o}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1
grep -E "passed|failed" $out/gpu_tests.log | tail -n 1
run() {
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact "$@" > $out/cfg3_bench_$name.json \
    2> $out/cfg3_bench_$name.err
  echo "$name $(cut -c1-90 $out/cfg3_bench_$name.json)"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['round_split'])" $out/cfg3_bench_$name.json
}
name=work; run
name=work_s0; run --opt nn_split_delta=0
export CLRRT_LIB=$GRAFT_REPO_ROOT/cl-rrt_amd/var_head/libclrrt.so
name=head_h50; run --opt nn_walk_hscale=50
unset CLRRT_LIB
name=work2; run
echo done
