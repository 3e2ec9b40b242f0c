# Round 5, first GPU session: the whole GPU suite (incl. the new full-size deferred-tree oracle tests) and one
# default cfg3 bench line.  Usage (repo root on the GPU box): bash tools/gpu_r05a.sh <tag>
set -e
tag=${1:-r05a}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread --maxfail=4 > $out/gpu_tests.log 2>&1 || rc=$?
# test failures (1) go on to the bench; a fault, abort or time limit ends the call here
if [ "${rc:-0}" -gt 1 ]; then echo "pytest rc=$rc"; exit $rc; fi
timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 > $out/cfg3_bench.json 2> $out/cfg3_bench.err
CLRRT_OPTS_AB="nn_walk_index=0;nn_walk_index=1;nn_walk_index=2;nn_walk_index=0" timeout -k 10 300 python3 -u tools/nn_large.py 1.0 3.5 8 16 > $out/nn_large_index_ab.txt 2>&1
