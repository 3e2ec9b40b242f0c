# Round-4 deferred-sample check on the GPU box: the BATCH parity tests (deferred and plain) and a cfg3 bench
# per defer_steps value.  Usage (repo root on the GPU box): bash tools/gpu_defer.sh <tag> "<T values>"
set -e
tag=${1:-d}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "deferred or batch_mode or pipelined" > $out/tests.log 2>&1
tail -n 3 $out/tests.log
for T in ${2:-0 128}; do
  timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-exact --no-sync --defer-steps $T \
    > $out/cfg3_T$T.json 2> $out/cfg3_T$T.err
  python3 -c "import json; d=json.loads(open('$out/cfg3_T$T.json').read().strip().splitlines()[-1]); print('T', $T, 'nodes/s', round(d['value']), 'frac', round(d['roofline']['frac'],4), 'roll ms', round(d['roofline']['avg_launch_ms'],3), 'deferred', d['config']['samples_deferred'], 'nn ms', round(d['kernel_ms']['nn']), 'roll total', round(d['kernel_ms']['rollout']))"
done
