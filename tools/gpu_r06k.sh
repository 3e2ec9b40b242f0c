# Round 6: the 3D walk index's heading axis scale (option nn_walk_hscale, percent of rho per radian): the walk alone on
# the 2.8 M-node tree and cfg3 bench lines.
# Usage (repo root on the GPU box): bash tools/gpu_r06k.sh <tag>
set -e
tag=${1:-r06k}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for h in 25 50 100 200; do
  CLRRT_OPTS=nn_walk_hscale=$h timeout -k 10 200 python3 -u tools/nn_large.py 2.8 > $out/nn_large_h$h.txt 2>&1
  grep mixed $out/nn_large_h$h.txt
done
for h in 50 100 25 200; do
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact --opt nn_walk_hscale=$h \
    > $out/cfg3_bench_h$h.json 2> $out/cfg3_bench_h$h.err
  echo "h$h $(cut -c1-90 $out/cfg3_bench_h$h.json)"
done
echo done
