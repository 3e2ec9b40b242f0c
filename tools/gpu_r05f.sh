# Round 5: EXACT fix-ups with the refined tie rule -- parity (EXACT tree tests, reference fixtures, Timer loop)
# then the fix-up statistics and EXACT throughput on cfg3.
set -e
tag=${1:-r05f}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_tree.py tests/test_native_timer_loop.py \
  tests/test_native_capi.py tests/test_native_plan_motion.py tests/test_replan.py -m gpu -k "exact or ref or timer or native or replan or budget" \
  -v -s --timeout 600 --timeout-method thread --maxfail=4 > $out/gpu_tests.log 2>&1 || rc=$?
if [ "${rc:-0}" -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 300 python3 -u tools/exact_fixup_stats.py 2000 > $out/exact_fixup_stats.txt 2>&1
