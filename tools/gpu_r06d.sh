# Round 6, fourth GPU session: the whole GPU suite on the build with the walk compiled without machine LICM (no
# scratch spills) and the round's resets folded; the walk without / with machine LICM on 2.8 and 16 M-node trees
# (tools/nn_large.py, CLRRT_LIB = the A/B build), cfg3 bench lines of both, the walk audit (non-member classes) and a
# kernel trace for the round timeline.
# Usage (repo root on the GPU box): bash tools/gpu_r06d.sh <tag>
set -e
tag=${1:-r06d}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 600 --timeout-method thread > $out/gpu_tests.log 2>&1
grep -E "passed|failed" $out/gpu_tests.log | tail -n 1
timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact > $out/cfg3_bench.json 2> $out/cfg3_bench.err
cut -c1-120 $out/cfg3_bench.json
CLRRT_LIB=cl-rrt_amd/var_licm/libclrrt.so timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact \
  > $out/cfg3_bench_licm.json 2> $out/cfg3_bench_licm.err
cut -c1-120 $out/cfg3_bench_licm.json
timeout -k 10 400 python3 -u tools/nn_large.py 2.8 16 > $out/nn_large.txt 2>&1
CLRRT_LIB=cl-rrt_amd/var_licm/libclrrt.so timeout -k 10 400 python3 -u tools/nn_large.py 2.8 16 > $out/nn_large_licm.txt 2>&1
timeout -k 10 300 python3 -u tools/walk_audit.py 1.1 2.8 > $out/walk_audit.txt 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o p -- python3 -u bench.py \
  --steps 2 --warmup 1 --no-cpu --no-exact --no-sync > $out/trace_bench.json 2> $out/trace_bench.err
gzip -f $out/trace/p_kernel_trace.csv
echo done
