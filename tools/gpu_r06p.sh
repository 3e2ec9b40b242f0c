# Round 6: hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4) against the lag-2 round's four streams
# (main and merge at high priority, two walk streams at low): cfg3 bench lines at 4 / 8 / 16 queues.
# Usage (repo root on the GPU box): bash tools/gpu_r06p.sh <tag>
set -e
tag=${1:-r06p}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() {
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact "$@" > $out/cfg3_bench_$name.json \
    2> $out/cfg3_bench_$name.err
  echo "$name $(cut -c1-90 $out/cfg3_bench_$name.json)"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['round_split'])" $out/cfg3_bench_$name.json
}
name=q4; run
GPU_MAX_HW_QUEUES=8 name=q8; export GPU_MAX_HW_QUEUES=8; run
export GPU_MAX_HW_QUEUES=16; name=q16; run
export GPU_MAX_HW_QUEUES=2; name=q2; run
unset GPU_MAX_HW_QUEUES
name=q4b; run
echo done
