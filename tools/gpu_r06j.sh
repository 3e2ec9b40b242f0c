# Round 6: the whole GPU suite with the new walk defaults (index kind 5, 8 walk waves per CU), the default cfg3 bench
# line, its kernel trace (round timeline) and the rollout lane-utilisation split (diagnostics build var_lane).
# Usage (repo root on the GPU box): bash tools/gpu_r06j.sh <tag>
set -e
tag=${1:-r06j}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1
grep -E "passed|failed" $out/gpu_tests.log | tail -n 1
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact > $out/cfg3_bench.json 2> $out/cfg3_bench.err
cut -c1-100 $out/cfg3_bench.json
CLRRT_LIB=cl-rrt_amd/var_lane/libclrrt.so timeout -k 10 300 python3 -u tools/lane_stats.py > $out/lane_stats.txt 2>&1
cat $out/lane_stats.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o p -- python3 -u bench.py \
  --steps 2 --warmup 1 --no-cpu --no-exact --no-sync > $out/trace_bench.json 2> $out/trace_bench.err
gzip -f $out/trace/p_kernel_trace.csv
echo done
