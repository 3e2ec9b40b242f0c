# Round-6 evidence on one GPU box for the final build: PMC FETCH/WRITE passes (cfg3, cfg2), SQ passes of the rollout
# kernel (wave states; VALU lane utilisation) and of the walk (a full 2 s query, so the large-tree format runs), a
# kernel-trace --stats profile of a cfg3 bench, the default bench line (CPU baselines and EXACT included) and the
# cfg2 / cfg5 lines.  Every summary records the sources' fingerprint (bench.py picks the pass of its own build).
# Part A (counters and trace; part B: tools/gpu_final6b.sh).
# Usage (repo root on the GPU box): bash tools/gpu_final6.sh <tag>
set -e
tag=${1:-r06zz}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
b1="bench.py --steps 1 --warmup 0 --no-cpu --no-exact --no-sync"
for cfg in cfg3 cfg2; do
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "k_roll_|k_walk_search" --output-format csv \
      -d $out/pmc_${cfg}_$c -o p -- python3 -u $b1 --config $cfg > $out/pmc_${cfg}_$c.log 2>&1
  done
  python3 tools/summarize_pmc.py $out/pmc_${cfg}_WRITE_SIZE/p_counter_collection.csv > $out/${cfg}_pmc_write.json
  python3 tools/summarize_pmc.py $out/pmc_${cfg}_FETCH_SIZE/p_counter_collection.csv > $out/${cfg}_pmc_fetch.json
  rm -f $out/pmc_${cfg}_*/p_counter_collection.csv
done
echo pmc done
g1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU"
g2="SQ_WAVES SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_BRANCH"
timeout -s KILL 200 rocprofv3 --pmc $g1 --kernel-include-regex "k_roll_run" --output-format csv -d $out/roll_sq -o p \
  -- python3 -u $b1 --horizon-ms 1000 > $out/roll_sq.log 2>&1
python3 tools/summarize_pmc.py $out/roll_sq/p_counter_collection.csv > $out/cfg3_roll_sq.json
timeout -s KILL 200 rocprofv3 --pmc $g2 --kernel-include-regex "k_roll_run" --output-format csv -d $out/roll_mix -o p \
  -- python3 -u $b1 --horizon-ms 1000 > $out/roll_mix.log 2>&1
python3 tools/summarize_pmc.py $out/roll_mix/p_counter_collection.csv > $out/cfg3_roll_mix.json
timeout -s KILL 200 rocprofv3 --pmc $g1 --kernel-include-regex "k_walk_search" --output-format csv -d $out/walk_sq -o p \
  -- python3 -u $b1 > $out/walk_sq.log 2>&1
python3 tools/summarize_pmc.py $out/walk_sq/p_counter_collection.csv > $out/cfg3_walk_sq.json
rm -f $out/*/p_counter_collection.csv
echo sq done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o p -- python3 -u bench.py --steps 3 \
  --warmup 1 --no-cpu --no-exact --no-sync > $out/trace_bench.json 2> $out/trace_bench.err
gzip -f $out/trace/p_kernel_trace.csv
echo trace done
echo part A done
