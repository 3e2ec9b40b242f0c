# Round 6: the build with the 96-VGPR walk and the 2304-wave grid as defaults: the whole GPU suite, the walk alone at
# 2.8 / 16 M nodes, a cfg3 bench line.
# Usage (repo root on the GPU box): bash tools/gpu_r06t.sh <tag>
set -e
tag=${1:-r06t}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1
grep -E "passed|failed" $out/gpu_tests.log | tail -n 1
timeout -k 10 400 python3 -u tools/nn_large.py 2.8 16 > $out/nn_large.txt 2>&1
grep -E "M nodes|mixed" $out/nn_large.txt
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact > $out/cfg3_bench.json 2> $out/cfg3_bench.err
cut -c1-90 $out/cfg3_bench.json
echo done
