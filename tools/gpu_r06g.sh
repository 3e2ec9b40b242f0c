# Round 6: the whole GPU suite on the build whose rollout kernels are compiled without machine LICM; the walk audit
# with the run statistics; the walk index kind 5 (equal records in ref.back() order) against kind 3 on 2.8 / 16 M-node
# trees and in cfg3 bench lines.
# Usage (repo root on the GPU box): bash tools/gpu_r06g.sh <tag>
set -e
tag=${1:-r06g}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1
grep -E "passed|failed" $out/gpu_tests.log | tail -n 1
timeout -k 10 300 python3 -u tools/walk_audit.py 1.1 2.8 > $out/walk_audit.txt 2>&1
for k in 3 5; do
  CLRRT_OPTS=nn_walk_index=$k timeout -k 10 400 python3 -u tools/nn_large.py 2.8 16 > $out/nn_large_k$k.txt 2>&1
done
for k in 3 5; do
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact --opt nn_walk_index=$k \
    > $out/cfg3_bench_k$k.json 2> $out/cfg3_bench_k$k.err
  cut -c1-100 $out/cfg3_bench_k$k.json
done
echo done
