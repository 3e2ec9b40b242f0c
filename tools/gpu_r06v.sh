# Round 6: the appended-node search started after the walk's main grid (option nn_delta_early, caps from k_walk_seed)
# instead of after its overflow split: the GPU suite, cfg3 bench lines off / on, and the list critical path of a trace.
# Usage (repo root on the GPU box): bash tools/gpu_r06v.sh <tag>
set -e
tag=${1:-r06v}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1
grep -E "passed|failed" $out/gpu_tests.log | tail -n 1
run() {
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact "$@" > $out/cfg3_bench_$name.json \
    2> $out/cfg3_bench_$name.err
  echo "$name $(cut -c1-90 $out/cfg3_bench_$name.json)"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['round_split'])" $out/cfg3_bench_$name.json
}
name=early1; run
name=early0; run --opt nn_delta_early=0
name=early1b; run
name=early1_split; run --opt nn_split_delta=1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o p -- python3 -u bench.py \
  --steps 2 --warmup 1 --no-cpu --no-exact --no-sync > $out/trace_bench.json 2> $out/trace_bench.err
python3 tools/list_crit.py $out/trace/p_kernel_trace.csv > $out/list_crit.txt
cat $out/list_crit.txt
gzip -f $out/trace/p_kernel_trace.csv
echo done
