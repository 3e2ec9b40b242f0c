set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcw
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --kernel-include-regex "k_walk_search" --output-format csv -d gpurun_out/pmcw/a -o a -- python3 -u tools/nn_walk_check.py 2000 > gpurun_out/pmcw/a.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-include-regex "k_walk_search" --output-format csv -d gpurun_out/pmcw/b -o b -- python3 -u tools/nn_walk_check.py 2000 > gpurun_out/pmcw/b.log 2>&1
