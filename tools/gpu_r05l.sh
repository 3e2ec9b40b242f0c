# Round 5: branched trigonometry for sparse waves (CLRRT_SPARSE_TRIG) and the partial std::sort replay of tied EXACT lists -- parity, then the lone step
# latency, EXACT throughput and the cfg3 bench against the build without it (cl-rrt_amd/prof_ab).
set -e
tag=${1:-r05l}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_tree.py tests/test_native_capi.py tests/test_replan.py -m gpu -x \
  -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
timeout -k 10 200 python3 -u tools/step_latency.py > $out/step_latency_sparse.txt 2>&1
CLRRT_LIB=cl-rrt_amd/prof_ab/libclrrt.so timeout -k 10 200 python3 -u tools/step_latency.py > $out/step_latency_base.txt 2>&1
timeout -k 10 200 python3 -u tools/exact_fixup_stats.py 2000 default > $out/exact_sparse.txt 2>&1
CLRRT_LIB=cl-rrt_amd/prof_ab/libclrrt.so timeout -k 10 200 python3 -u tools/exact_fixup_stats.py 2000 default > $out/exact_base.txt 2>&1
timeout -k 10 300 python3 -u bench.py --no-cpu > $out/bench_sparse.json 2> $out/bench_sparse.err
CLRRT_LIB=cl-rrt_amd/prof_ab/libclrrt.so timeout -k 10 300 python3 -u bench.py --no-cpu > $out/bench_base.json 2> $out/bench_base.err
echo done
