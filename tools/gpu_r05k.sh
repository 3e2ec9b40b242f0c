# Round 5: SQ instruction mix of a lone rollout (tools/lone_sq.py): k_rollout of the longest cfg3 rollout alone,
# EXACT iterations at width 1 (k_roll_run).  Two passes of 8 SQ counters each.
set -e
tag=${1:-r05k}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 200 python3 -u tools/lone_sq.py > $out/lone_plain.txt 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM \
  --kernel-include-regex "k_roll" --output-format csv -d $out/sq1 -o p -- python3 -u tools/lone_sq.py > $out/sq1.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS \
  --kernel-include-regex "k_roll" --output-format csv -d $out/sq2 -o p -- python3 -u tools/lone_sq.py > $out/sq2.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/exact_prof -o p \
  -- python3 -u tools/exact_fixup_stats.py 1000 default > $out/exact_rocprof.txt 2>&1
echo done
