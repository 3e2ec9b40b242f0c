# Round 5 final profiling session of the current build: tools/gpu_r05b.sh's passes (rocprof kernel stats, PMC FETCH/WRITE
# cfg3 + cfg2, walk and rollout SQ passes with the sources' fingerprint), the round's critical path, and the rollout step
# latency / phases (diagnostics build cl-rrt_amd/prof for the phases).
set -e
tag=${1:-r05t}
build=${2:-unknown}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/$tag
bash tools/gpu_r05b.sh $tag $build
python3 tools/round_crit.py $out/prof/p_kernel_trace.csv > $out/cfg3_round_crit.txt
timeout -k 10 200 python3 -u tools/step_latency.py > $out/step_latency.txt 2>&1
CLRRT_LIB=cl-rrt_amd/prof/libclrrt.so timeout -k 10 300 python3 -u tools/step_phases.py > $out/step_phases.txt 2>&1
echo done
