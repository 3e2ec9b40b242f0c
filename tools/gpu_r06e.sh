# Round 6: A/B of the rollout kernels compiled without machine LICM (256 VGPRs + 64 AGPRs instead of + 157, so a
# 128-register walk wave fits beside a rollout wave on its SIMD): cfg3 bench lines (BATCH + EXACT) and the rollout
# step latency (tools/step_latency.py) of both builds.
# Usage (repo root on the GPU box): bash tools/gpu_r06e.sh <tag>
set -e
tag=${1:-r06e}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base rollnolicm; do
  lib=cl-rrt_amd/libclrrt.so
  [ $v = rollnolicm ] && lib=cl-rrt_amd/var_rollnolicm/libclrrt.so
  CLRRT_LIB=$lib timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 1 --no-cpu > $out/cfg3_bench_$v.json \
    2> $out/cfg3_bench_$v.err
  cut -c1-120 $out/cfg3_bench_$v.json
  CLRRT_LIB=$lib timeout -k 10 200 python3 -u tools/step_latency.py > $out/step_latency_$v.txt 2>&1
done
for v in base rollnolicm; do
  lib=cl-rrt_amd/libclrrt.so
  [ $v = rollnolicm ] && lib=cl-rrt_amd/var_rollnolicm/libclrrt.so
  CLRRT_LIB=$lib timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact \
    > $out/cfg3_bench2_$v.json 2> $out/cfg3_bench2_$v.err
  cut -c1-120 $out/cfg3_bench2_$v.json
done
echo done
