# Round 6: the walk's persistent grid and index kind re-tuned for the 320-register rollout kernels (cfg3 bench lines):
# kind 5 with 6 .. 9 walk waves per CU, the old defaults (kind 3, 10 per CU) as the reference.
# Usage (repo root on the GPU box): bash tools/gpu_r06i.sh <tag>
set -e
tag=${1:-r06i}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact "$@" > $out/cfg3_bench_$name.json \
    2> $out/cfg3_bench_$name.err
  echo "$name $(cut -c1-90 $out/cfg3_bench_$name.json)"
}
name=k3w2560; run --opt nn_walk_index=3 --opt nn_walk_waves=2560
name=k5w2048; run --opt nn_walk_index=5 --opt nn_walk_waves=2048
name=k5w1792; run --opt nn_walk_index=5 --opt nn_walk_waves=1792
name=k5w1536; run --opt nn_walk_index=5 --opt nn_walk_waves=1536
name=k5w2304; run --opt nn_walk_index=5 --opt nn_walk_waves=2304
name=k5w2048rb128; run --opt nn_walk_index=5 --opt nn_walk_waves=2048 --opt roll_blocks=128
name=k3w2048; run --opt nn_walk_index=3 --opt nn_walk_waves=2048
name=k5w2048b; run --opt nn_walk_index=5 --opt nn_walk_waves=2048
echo done
