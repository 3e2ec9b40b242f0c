# Round 5: the overflow split waves share their pruning bound -- walk parity (brute force, overflow records,
# cfg3 bench-size tree, the bench settings' deferred tree), then the walk time on 4.7 M / 16 M node trees
# against the build without sharing (cl-rrt_amd/prof_ab), then the bench line.
set -e
tag=${1:-r05j}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_full_size_parity.py -m gpu \
  -k "walk or cfg3 or bench_settings" -v -s --timeout 900 --timeout-method thread -x > $out/gpu_tests.log 2>&1
timeout -k 10 300 python3 -u tools/nn_large.py 4.7 16 > $out/nn_large_share.txt 2>&1
CLRRT_LIB=cl-rrt_amd/prof_ab/libclrrt.so timeout -k 10 300 python3 -u tools/nn_large.py 4.7 16 > $out/nn_large_noshare.txt 2>&1
timeout -k 10 300 python3 -u bench.py > $out/bench.json 2> $out/bench.err
