# Round-4 GPU session: the GPU suite (live log), then a cfg3 bench per defer_steps value.
# Usage (repo root on the GPU box): bash tools/gpu_r04.sh <tag> "<T values>" [tests|notests]
set -e
tag=${1:-r04}
out=gpurun_out/$tag
mkdir -p $out
if [ "${3:-tests}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || true
  tail -n 3 $out/gpu_tests.log
  grep -E "FAILED|ERROR" $out/gpu_tests.log | head -20 || true
fi
for T in ${2:-128}; do
  timeout -k 10 240 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-exact --no-sync --defer-steps $T \
    > $out/cfg3_T$T.json 2> $out/cfg3_T$T.err
  python3 -c "import json; d=json.loads(open('$out/cfg3_T$T.json').read().strip().splitlines()[-1]); print('T', $T, 'nodes/s', round(d['value']), 'frac', round(d['roofline']['frac'],4), 'roll ms', round(d['roofline']['avg_launch_ms'],3), 'deferred', d['config']['samples_deferred'], 'nn ms', round(d['kernel_ms']['nn']), 'roll total', round(d['kernel_ms']['rollout']), 'launches', d['kernel_ms']['launches'])"
done
