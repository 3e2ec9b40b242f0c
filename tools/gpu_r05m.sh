# Round 5: EXACT speculative rollouts one per wave (k_rollout SRC_SPEC, option exact_lone) -- EXACT parity tests,
# then EXACT throughput with exact_lone 1 / 0 and an EXACT kernel trace.
set -e
tag=${1:-r05m}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_tree.py tests/test_native_timer_loop.py \
  tests/test_native_capi.py tests/test_replan.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
timeout -k 10 200 python3 -u tools/exact_fixup_stats.py 2000 default exact_lone=1 > $out/exact_lone1.txt 2>&1
timeout -k 10 200 python3 -u tools/exact_fixup_stats.py 2000 default exact_lone=0 > $out/exact_lone0.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/exact_prof -o p \
  -- python3 -u tools/exact_fixup_stats.py 1000 default > $out/exact_rocprof.txt 2>&1
echo done
