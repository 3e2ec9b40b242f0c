# Round 6: blocks of the lag-2 appended-node search (option nn_delta_blocks in build var_db; default 2048), cfg3 lines.
# Usage (repo root on the GPU box): bash tools/gpu_r06zb.sh <tag>
set -e
tag=${1:-r06zb}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export CLRRT_LIB=$GRAFT_REPO_ROOT/cl-rrt_amd/var_db/libclrrt.so
run() {
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact "$@" > $out/cfg3_bench_$name.json \
    2> $out/cfg3_bench_$name.err
  echo "$name $(cut -c1-90 $out/cfg3_bench_$name.json)"
}
name=b2048; run
name=b1024; run --opt nn_delta_blocks=1024
name=b4096; run --opt nn_delta_blocks=4096
name=b8192; run --opt nn_delta_blocks=8192
name=b2048b; run
echo done
