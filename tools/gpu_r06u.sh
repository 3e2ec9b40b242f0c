# Round 6: the rollout grid schedule re-checked with the 96-VGPR walk (two walk waves beside each rollout wave): the
# default (7/8 .. 3/8 of the CUs as the tree grows) against fixed 96 / 128 / 160 / 192 blocks, cfg3 bench lines.
# Usage (repo root on the GPU box): bash tools/gpu_r06u.sh <tag>
set -e
tag=${1:-r06u}
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
name=rb96; run --opt roll_blocks=96
name=rb128; run --opt roll_blocks=128
name=rb160; run --opt roll_blocks=160
name=rb192; run --opt roll_blocks=192
name=default2; run
echo done
