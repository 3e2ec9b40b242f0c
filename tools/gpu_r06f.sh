# Round 6: (1) the walk with a table of known run keys (WALK_RUNS) -- its parity tests, then the walk alone on 2.8 /
# 16 M-node trees against the previous walk (var_walk0), (2) cfg3 bench lines of the default build, the previous
# walk and the rollout kernels without machine LICM (var_rollnolicm), (3) EXACT and the step latency of the default
# build and var_rollnolicm.
# Usage (repo root on the GPU box): bash tools/gpu_r06f.sh <tag>
set -e
tag=${1:-r06f}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_parity.py -m gpu -v \
  -k "walk or nearest or pipelined or deferred or bench_size or late_query" --timeout 600 --timeout-method thread \
  > $out/walk_tests.log 2>&1
grep -E "passed|failed" $out/walk_tests.log | tail -n 1
timeout -k 10 400 python3 -u tools/nn_large.py 2.8 16 > $out/nn_large.txt 2>&1
CLRRT_LIB=cl-rrt_amd/var_walk0/libclrrt.so timeout -k 10 400 python3 -u tools/nn_large.py 2.8 16 > $out/nn_large_walk0.txt 2>&1
for v in base walk0 rollnolicm; do
  lib=cl-rrt_amd/libclrrt.so
  [ $v = walk0 ] && lib=cl-rrt_amd/var_walk0/libclrrt.so
  [ $v = rollnolicm ] && lib=cl-rrt_amd/var_rollnolicm/libclrrt.so
  CLRRT_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact \
    > $out/cfg3_bench_$v.json 2> $out/cfg3_bench_$v.err
  cut -c1-100 $out/cfg3_bench_$v.json
done
for v in base rollnolicm; do
  lib=cl-rrt_amd/libclrrt.so
  [ $v = rollnolicm ] && lib=cl-rrt_amd/var_rollnolicm/libclrrt.so
  CLRRT_LIB=$lib timeout -k 10 200 python3 -u tools/step_latency.py > $out/step_latency_$v.txt 2>&1
  CLRRT_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 --no-cpu --no-sync \
    > $out/cfg3_exact_$v.json 2> $out/cfg3_exact_$v.err
done
echo done
