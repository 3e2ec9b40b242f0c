# Round 5: EXACT speculative rollouts one per wave on k_rollout (option exact_lone) after the rollout kernels' parameter
# change -- EXACT parity, EXACT throughput exact_lone 1 / 0 (x2 each, alternating), 16 GPU replicas.
set -e
tag=${1:-r05s}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_tree.py tests/test_native_timer_loop.py \
  tests/test_native_capi.py -m gpu -x -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python3 -u tools/exact_fixup_stats.py 2000 default exact_lone=1 >> $out/exact_lone1.txt 2>&1
  timeout -k 10 200 python3 -u tools/exact_fixup_stats.py 2000 default exact_lone=0 >> $out/exact_lone0.txt 2>&1
done
timeout -k 10 300 python3 -u tools/exact_replicas.py 16 > $out/exact_replicas.txt 2>&1
echo done
