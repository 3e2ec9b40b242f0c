# Round 6: with the rollout kernels at 320 registers per lane a walk wave fits beside a rollout wave, so the schedule
# tuned for the old footprint is re-checked: the rollout grid width (default: 7/8 .. 3/8 of the CUs as the tree
# grows; fixed widths) and the walk's persistent grid (default 10 waves per CU), cfg3 bench lines.
# Usage (repo root on the GPU box): bash tools/gpu_r06h.sh <tag>
set -e
tag=${1:-r06h}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact "$@" > $out/cfg3_bench_$name.json \
    2> $out/cfg3_bench_$name.err
  echo "$name $(cut -c1-90 $out/cfg3_bench_$name.json)"
}
name=default; run
name=rb128; run --opt roll_blocks=128
name=rb160; run --opt roll_blocks=160
name=rb192; run --opt roll_blocks=192
name=ww3072; run --opt nn_walk_waves=3072
name=ww3584; run --opt nn_walk_waves=3584
name=ww2048; run --opt nn_walk_waves=2048
name=default2; run
echo done
