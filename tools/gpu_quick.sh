# One A/B iteration on the GPU box: the GPU suite, a short cfg3 bench, the rollout timeline (diagnostics build).
# Usage (repo root on the GPU box): bash tools/gpu_quick.sh <tag> [tests|notests]
set -e
tag=${1:-q}
out=gpurun_out/$tag
mkdir -p $out
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
  tail -n 2 $out/gpu_tests.log
fi
timeout -k 10 200 python3 -u bench.py --steps 4 --warmup 1 --no-cpu > $out/cfg3_bench.json 2> $out/cfg3_bench.err
python3 -c "import json,sys; d=json.loads(open('$out/cfg3_bench.json').read().strip().splitlines()[-1]); print('cfg3', d['value'], 'frac', d['roofline']['frac'], 'roll ms', d['roofline']['avg_launch_ms'], 'exact', d['exact_mode']['value'])"
CLRRT_LIB=cl-rrt_amd/prof/libclrrt.so timeout -k 10 200 python3 -u tools/roll_phases.py 1000 > $out/roll_phases.txt 2>&1
grep -E "single round|sparse|pipelined" $out/roll_phases.txt
