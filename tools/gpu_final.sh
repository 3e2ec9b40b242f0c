# Round-end evidence on one GPU box: the GPU suite, PMC FETCH/WRITE passes (cfg3, cfg2), a kernel-trace --stats
# profile of a cfg3 bench, the default bench line (CPU baselines included) and the cfg2 / cfg5 lines.
# Usage (repo root on the GPU box): bash tools/gpu_final.sh <tag> [notests]
set -e
tag=${1:-r04final}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1
  tail -n 1 $out/gpu_tests.log
fi
for cfg in cfg3 cfg2; do
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex "k_roll_|k_walk_search" --output-format csv \
      -d $out/pmc_${cfg}_$c -o p -- python3 -u bench.py --config $cfg --steps 1 --warmup 0 --no-cpu --no-exact --no-sync \
      --horizon-ms 500 > $out/pmc_${cfg}_$c.log 2>&1
  done
  python3 tools/summarize_pmc.py $out/pmc_${cfg}_WRITE_SIZE/p_counter_collection.csv > $out/${cfg}_pmc_write.json
  python3 tools/summarize_pmc.py $out/pmc_${cfg}_FETCH_SIZE/p_counter_collection.csv > $out/${cfg}_pmc_fetch.json
  rm -f $out/pmc_${cfg}_*/p_counter_collection.csv
done
echo pmc done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o p -- python3 -u bench.py --steps 3 \
  --warmup 1 --no-cpu --no-exact --no-sync > $out/trace_bench.json 2> $out/trace_bench.err
rm -f $out/trace/p_kernel_trace.csv
echo trace done
timeout -k 10 400 python3 -u bench.py > $out/cfg3_bench.json 2> $out/cfg3_bench.err
cut -c1-200 $out/cfg3_bench.json
timeout -k 10 200 python3 -u bench.py --config cfg2 --steps 10 --warmup 2 --no-cpu > $out/cfg2_bench.json 2> $out/cfg2_bench.err
timeout -k 10 200 python3 -u bench.py --config cfg5 --steps 5 --warmup 1 --no-cpu > $out/cfg5_bench.json 2> $out/cfg5_bench.err
echo all done
