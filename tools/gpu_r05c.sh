# Round 5: the Timer-loop drop-in test, and the walk index A/B with the ang_par octant kept on top (kinds 3 / 4).
# Usage (repo root on the GPU box): bash tools/gpu_r05c.sh <tag>
set -e
tag=${1:-r05c}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_native_timer_loop.py tests/test_native_capi.py -m gpu -v -s --timeout 300 --timeout-method thread > $out/timer_tests.log 2>&1
CLRRT_OPTS_AB="nn_walk_index=0;nn_walk_index=3;nn_walk_index=4;nn_walk_index=0" timeout -k 10 300 python3 -u tools/nn_large.py 1.0 2.5 4 16 > $out/nn_large_index_ab2.txt 2>&1
