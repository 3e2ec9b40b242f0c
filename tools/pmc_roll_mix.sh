# rocprofv3 PMC passes over the rollout kernel's instruction mix (one counter group per run) on a fixed
# cfg3 round (tools/roll_fixed.py).  Output: gpurun_out/pmcm/<group>/
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcm
g1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_WAVE_CYCLES SQ_WAIT_INST_ANY"
g2="SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"
g3="SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM"
i=0
for g in "$g1" "$g2" "$g3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $g --kernel-include-regex "k_roll_run" --output-format csv -d gpurun_out/pmcm/g$i -o p \
    -- python3 -u tools/roll_fixed.py 500 2 > gpurun_out/pmcm/g$i.log 2>&1
done
