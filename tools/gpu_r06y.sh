# Round 6 final build (lane order adopted): the whole GPU suite, then part A of the final evidence (gpu_final6.sh).
# Usage (repo root on the GPU box): bash tools/gpu_r06y.sh <tag>
set -e
tag=${1:-r06zz}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1
grep -E "passed|failed" $out/gpu_tests.log | tail -n 1
bash tools/gpu_final6.sh $tag
