# Round 6: longest-first samples in the persistent walk's eighths (option nn_walk_lpt): the walk parity tests with it on (the build default),
# the walk alone on 2.8 M nodes, cfg3 bench lines off / on.
# Usage (repo root on the GPU box): bash tools/gpu_r06q.sh <tag>
set -e
tag=${1:-r06q}
out=gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_full_size_parity.py tests/test_gpu_parity.py -m gpu -v -s \
  --timeout 300 --timeout-method thread -k "walk or brute or bench_size or late_query or bench_settings or deferred or pipelined" \
  > $out/gpu_tests_lpt.log 2>&1
grep -E "passed|failed" $out/gpu_tests_lpt.log | tail -n 1
for v in 0 1; do
  CLRRT_OPTS=nn_walk_lpt=$v timeout -k 10 200 python3 -u tools/nn_large.py 2.8 > $out/nn_large_lpt$v.txt 2>&1
  grep -E "mixed" $out/nn_large_lpt$v.txt
done
run() {
  timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-exact "$@" > $out/cfg3_bench_$name.json \
    2> $out/cfg3_bench_$name.err
  echo "$name $(cut -c1-90 $out/cfg3_bench_$name.json)"
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['round_split'])" $out/cfg3_bench_$name.json
}
name=lpt0; run --opt nn_walk_lpt=0
name=lpt1; run
name=lpt0b; run --opt nn_walk_lpt=0
name=lpt1b; run
echo done
