# Round 5: EXACT fix-up prefetch (option exact_prefetch) -- EXACT parity, then EXACT throughput with the prefetch on / off
# and an EXACT kernel trace.
set -e
tag=${1:-r05n}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
export CLRRT_XF_REPORT=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_tree.py tests/test_native_timer_loop.py \
  -m gpu -k "exact or ref or timer or device or fixup" -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
timeout -k 10 200 python3 -u tools/exact_fixup_stats.py 2000 default exact_prefetch=1 > $out/exact_pf1.txt 2>&1
timeout -k 10 200 python3 -u tools/exact_fixup_stats.py 2000 default exact_prefetch=0 > $out/exact_pf0.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/exact_prof -o p \
  -- python3 -u tools/exact_fixup_stats.py 1000 default > $out/exact_rocprof.txt 2>&1
echo done
