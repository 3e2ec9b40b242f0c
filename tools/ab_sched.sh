# A/B of LLVM scheduler strategies for the rollout/walk kernels on a fixed cfg3 round (build the variants first with tools/variant.sh ilp|memc|bias0 ...).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 120 python3 -u tools/roll_fixed.py r40 8 > gpurun_out/ab/base.log 2>&1
for v in ilp memc bias0; do
  CLRRT_LIB=build/$v/libclrrt.so timeout -k 10 120 python3 -u tools/roll_fixed.py r40 8 > gpurun_out/ab/$v.log 2>&1
done
timeout -k 10 120 python3 -u tools/roll_fixed.py r40 8 > gpurun_out/ab/base2.log 2>&1
echo done
