# Round 5: EXACT rounds with fix-ups (parity: the EXACT tree tests, the reference fixtures incl. the 2435-node tree,
# the Timer loop), the walk index default (kind 3) on the walk parity tests, and a cfg3 bench line.
# Usage (repo root on the GPU box): bash tools/gpu_r05d.sh <tag>
set -e
tag=${1:-r05d}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_tree.py tests/test_native_timer_loop.py \
  tests/test_native_capi.py tests/test_native_plan_motion.py -m gpu -v -s --timeout 600 --timeout-method thread \
  --maxfail=4 > $out/gpu_tests.log 2>&1 || rc=$?
if [ "${rc:-0}" -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --no-cpu > $out/cfg3_bench.json 2> $out/cfg3_bench.err
