# Round-6 evidence on one GPU box for the final build: PMC FETCH/WRITE passes (cfg3, cfg2), SQ passes of the rollout
# kernel (wave states; VALU lane utilisation) and of the walk (a full 2 s query, so the large-tree format runs), a
# kernel-trace --stats profile of a cfg3 bench, the default bench line (CPU baselines and EXACT included) and the
# cfg2 / cfg5 lines.  Every summary records the sources' fingerprint (bench.py picks the pass of its own build).
# Part B (bench lines and smoke; part A: tools/gpu_final6.sh).
# Usage (repo root on the GPU box): bash tools/gpu_final6b.sh <tag>
set -e
tag=${1:-r06zz}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python3 -u bench.py > $out/cfg3_bench.json 2> $out/cfg3_bench.err
cut -c1-200 $out/cfg3_bench.json
timeout -k 10 200 python3 -u bench.py --config cfg2 --steps 10 --warmup 2 --no-cpu > $out/cfg2_bench.json 2> $out/cfg2_bench.err
timeout -k 10 200 python3 -u bench.py --config cfg5 --steps 5 --warmup 1 --no-cpu > $out/cfg5_bench.json 2> $out/cfg5_bench.err
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
tail -n 2 $out/smoke.log
echo all done
