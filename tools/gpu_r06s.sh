# Round 6: the 96-VGPR walk build (var_w5) around its best grid of r06r (2560 waves): 2304 / 2560 / 2816, each twice,
# cfg3 bench lines.
# Usage (repo root on the GPU box): bash tools/gpu_r06s.sh <tag>
set -e
tag=${1:-r06s}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact "$@" > $out/cfg3_bench_$name.json \
    2> $out/cfg3_bench_$name.err
  echo "$name $(cut -c1-90 $out/cfg3_bench_$name.json)"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['round_split'])" $out/cfg3_bench_$name.json
}
export CLRRT_LIB=$GRAFT_REPO_ROOT/cl-rrt_amd/var_w5/libclrrt.so
name=w5_2304; run --opt nn_walk_waves=2304
name=w5_2560; run --opt nn_walk_waves=2560
name=w5_2816; run --opt nn_walk_waves=2816
name=w5_2304b; run --opt nn_walk_waves=2304
name=w5_2560b; run --opt nn_walk_waves=2560
name=w5_2816b; run --opt nn_walk_waves=2816
echo done
