# Round 6: the walk kernels at 96 VGPRs (CLRRT_WALK_WAVES 5, var_w5: two walk waves fit on a SIMD beside a 320-register
# rollout wave, at 64-128 B/lane of scratch) against the default 128, with 8 / 10 / 12 walk waves per CU; cfg3 lines.
# Usage (repo root on the GPU box): bash tools/gpu_r06r.sh <tag>
set -e
tag=${1:-r06r}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact "$@" > $out/cfg3_bench_$name.json \
    2> $out/cfg3_bench_$name.err
  echo "$name $(cut -c1-90 $out/cfg3_bench_$name.json)"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['round_split'])" $out/cfg3_bench_$name.json
}
name=default; run
export CLRRT_LIB=$GRAFT_REPO_ROOT/cl-rrt_amd/var_w5/libclrrt.so
name=w5_2048; run
name=w5_2560; run --opt nn_walk_waves=2560
name=w5_3072; run --opt nn_walk_waves=3072
unset CLRRT_LIB
name=default2; run
echo done
