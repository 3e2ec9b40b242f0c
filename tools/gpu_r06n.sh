# Round 6: the committed build (var_head) against the working build, cfg3 bench lines in one session: does the working
# build's rollout kernel (4.1 vs 2.6 ms per round in r06l / r06m) come from the build or from the box?
# Usage (repo root on the GPU box): bash tools/gpu_r06n.sh <tag>
set -e
tag=${1:-r06n}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact "$@" > $out/cfg3_bench_$name.json \
    2> $out/cfg3_bench_$name.err
  echo "$name $(cut -c1-90 $out/cfg3_bench_$name.json)"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['round_split'])" $out/cfg3_bench_$name.json
}
export CLRRT_LIB=$GRAFT_REPO_ROOT/cl-rrt_amd/var_head/libclrrt.so
name=head; run
name=head_h50; run --opt nn_walk_hscale=50
unset CLRRT_LIB
name=work_s0h100; run --opt nn_split_delta=0 --opt nn_walk_hscale=100
name=work; run
export CLRRT_LIB=$GRAFT_REPO_ROOT/cl-rrt_amd/var_head/libclrrt.so
name=head2; run
echo done
