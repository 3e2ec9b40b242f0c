# Round 6: the split appended-node search (option nn_split_delta): the whole GPU suite (every lag-2 tree test runs
# it), then cfg3 bench lines with it off / on, and a kernel trace of the default build (round timeline).
# Usage (repo root on the GPU box): bash tools/gpu_r06l.sh <tag>
set -e
tag=${1:-r06l}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1
grep -E "passed|failed" $out/gpu_tests.log | tail -n 1
for v in 1 0 1; do
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact --opt nn_split_delta=$v \
    > $out/cfg3_bench_split$v.json 2> $out/cfg3_bench_split$v.err
  echo "split$v $(cut -c1-90 $out/cfg3_bench_split$v.json)"
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o p -- python3 -u bench.py \
  --steps 2 --warmup 1 --no-cpu --no-exact --no-sync > $out/trace_bench.json 2> $out/trace_bench.err
gzip -f $out/trace/p_kernel_trace.csv
echo done
