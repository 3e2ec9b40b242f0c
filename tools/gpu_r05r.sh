# Round 5: the query parameters in LDS in the rollout kernels (CLRRT_PARAMS_LDS) -- rollout parity, then the lone step
# latency, EXACT and the cfg3 bench against the build without it (cl-rrt_amd/prof_ab).
set -e
tag=${1:-r05r}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_ref_tree.py -m gpu -x \
  -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
timeout -k 10 200 python3 -u tools/step_latency.py > $out/step_latency_lds.txt 2>&1
CLRRT_LIB=cl-rrt_amd/prof_ab/libclrrt.so timeout -k 10 200 python3 -u tools/step_latency.py > $out/step_latency_reg.txt 2>&1
timeout -k 10 200 python3 -u tools/exact_fixup_stats.py 2000 default > $out/exact_lds.txt 2>&1
CLRRT_LIB=cl-rrt_amd/prof_ab/libclrrt.so timeout -k 10 200 python3 -u tools/exact_fixup_stats.py 2000 default > $out/exact_reg.txt 2>&1
timeout -k 10 300 python3 -u bench.py --no-cpu --no-exact > $out/bench_lds.json 2> $out/bench_lds.err
CLRRT_LIB=cl-rrt_amd/prof_ab/libclrrt.so timeout -k 10 300 python3 -u bench.py --no-cpu --no-exact > $out/bench_reg.json 2> $out/bench_reg.err
echo done
