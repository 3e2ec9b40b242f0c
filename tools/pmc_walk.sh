# PMC passes over the walk search of tools/nn_large.py (one tree size, argv $1 M nodes; output dir $2)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/${2:-pmcw}; mkdir -p $out
n=${1:-2.2}
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-include-regex "k_walk_search" --output-format csv -d $out/a -o a -- python3 -u tools/nn_large.py $n > $out/a.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM --kernel-include-regex "k_walk_search" --output-format csv -d $out/b -o b -- python3 -u tools/nn_large.py $n > $out/b.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-include-regex "k_walk_search" --output-format csv -d $out/c -o c -- python3 -u tools/nn_large.py $n > $out/c.log 2>&1
