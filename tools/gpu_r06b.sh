# Round 6, second GPU session: the walk's measured bound (tools/walk_audit.py at 1.1 / 2.8 / 16 M nodes), a kernel
# trace of two cfg3 queries kept for the main-stream timeline of a round (tools/round_timeline.py), the first SQ /
# FETCH / WRITE passes of the large-tree walk format (k_walk_search<1, ...>: a full 2 s query, trees past 1.3 M
# nodes) and the round split at smaller per-GPU batches (the strong-scaling projection of DESIGN.md section 7).
# Usage (repo root on the GPU box): bash tools/gpu_r06b.sh <tag>
set -e
tag=${1:-r06b}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 420 python3 -u tools/walk_audit.py 1.1 2.8 16 > $out/walk_audit.txt 2>&1
cat $out/walk_audit.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o p -- python3 -u bench.py \
  --steps 2 --warmup 1 --no-cpu --no-exact --no-sync > $out/trace_bench.json 2> $out/trace_bench.err
gzip -f $out/trace/p_kernel_trace.csv
echo trace done
w="--kernel-include-regex k_walk_search --output-format csv"
b="bench.py --steps 1 --warmup 0 --no-cpu --no-exact --no-sync"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_INSTS_VALU SQ_ACTIVE_INST_VALU $w -d $out/sq -o p -- python3 -u $b > $out/sq.log 2>&1
python3 tools/summarize_pmc.py $out/sq/p_counter_collection.csv > $out/cfg3_walk_sq.json
rm -f $out/sq/p_counter_collection.csv
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD \
  SQ_INSTS_FLAT SQ_INSTS_BRANCH $w -d $out/sq2 -o p -- python3 -u $b > $out/sq2.log 2>&1
python3 tools/summarize_pmc.py $out/sq2/p_counter_collection.csv > $out/cfg3_walk_sq2.json
rm -f $out/sq2/p_counter_collection.csv
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c --kernel-include-regex "k_roll_|k_walk_search" --output-format csv \
    -d $out/pmc_$c -o p -- python3 -u $b > $out/pmc_$c.log 2>&1
  python3 tools/summarize_pmc.py $out/pmc_$c/p_counter_collection.csv > $out/cfg3_pmc_$c.json
  rm -f $out/pmc_$c/p_counter_collection.csv
done
echo pmc done
for bb in 2048 4096 8192; do
  timeout -k 10 120 python3 -u bench.py --batch $bb --steps 2 --warmup 1 --no-cpu --no-exact --no-sync \
    > $out/cfg3_batch$bb.json 2> $out/cfg3_batch$bb.err
done
echo done
