# PMC passes over k_walk_search in a short cfg3 bench run (the bench line's roofline_walk reads the summaries):
# SQ wave-state counters, then FETCH_SIZE / WRITE_SIZE.  Usage (GPU box, repo root): bash tools/pmc_walk_bench.sh <out_dir>
set -e
out=${1:-gpurun_out/pmcwb}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p $out
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
  --kernel-include-regex "k_walk_search" --output-format csv -d $out/sq -o p -- python3 -u bench.py --steps 1 --warmup 0 \
  --no-cpu --no-exact --no-sync --horizon-ms 1000 > $out/sq.log 2>&1
python3 tools/summarize_pmc.py $out/sq/p_counter_collection.csv > $out/walk_sq.json
rm -f $out/sq/p_counter_collection.csv
