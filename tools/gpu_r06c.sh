# Round 6, third GPU session: the whole GPU suite on the build with the round's resets folded into one launch (and the
# walk's into its key kernel), the walk audit with the non-member classification (1.1 / 2.8 M nodes), a cfg3 bench
# line and a kernel trace for the round timeline (tools/round_timeline.py).
# Usage (repo root on the GPU box): bash tools/gpu_r06c.sh <tag>
set -e
tag=${1:-r06c}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1
tail -n 1 $out/gpu_tests.log
timeout -k 10 300 python3 -u tools/walk_audit.py 1.1 2.8 > $out/walk_audit.txt 2>&1
cat $out/walk_audit.txt
timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-exact > $out/cfg3_bench.json 2> $out/cfg3_bench.err
cut -c1-200 $out/cfg3_bench.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o p -- python3 -u bench.py \
  --steps 2 --warmup 1 --no-cpu --no-exact --no-sync > $out/trace_bench.json 2> $out/trace_bench.err
gzip -f $out/trace/p_kernel_trace.csv
echo done
