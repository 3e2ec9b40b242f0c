# Round 6, first GPU session: the changed tests (sharded exchange ABI 11, closing exchange, world-8 rehearsal, drop-in
# rand() check), a short cfg3 bench line (round split), and the 8-rank cfg4 strong-split rehearsal on one GPU (gloo).
# Usage (repo root on the GPU box): bash tools/gpu_r06a.sh <tag>
set -e
tag=${1:-r06a}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py tests/test_native_timer_loop.py -v -s --timeout 600 \
  --timeout-method thread > $out/gpu_tests.log 2>&1
tail -n 1 $out/gpu_tests.log
timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-exact > $out/cfg3_bench.json 2> $out/cfg3_bench.err
cut -c1-160 $out/cfg3_bench.json
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29561 bench.py --gpus 8 --dist-backend gloo --scaling strong --steps 2 --warmup 1 --no-cpu --no-exact \
  --max-nodes 3145728 > $out/cfg4_strong_8ranks_gloo.json 2> $out/cfg4_strong_8ranks_gloo.err
cut -c1-160 $out/cfg4_strong_8ranks_gloo.json
echo done
