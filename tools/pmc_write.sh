# FETCH_SIZE / WRITE_SIZE passes (one counter per run) for the rollout and walk kernels on a short cfg3 bench.
# Usage (GPU box, repo root): bash tools/pmc_write.sh <out_dir> [config]
set -e
out=${1:-gpurun_out/pmcw}
cfgname=${2:-cfg3}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p $out
for c in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex "k_roll_|k_walk_search" --output-format csv \
    -d $out/$c -o p -- python3 -u bench.py --config $cfgname --steps 1 --warmup 0 --no-cpu --no-exact --horizon-ms 500 \
    > $out/$c.log 2>&1
done
python3 tools/summarize_pmc.py $out/WRITE_SIZE/p_counter_collection.csv > $out/write.json; python3 tools/summarize_pmc.py $out/FETCH_SIZE/p_counter_collection.csv > $out/fetch.json
