# A/B of library builds on one box with a short cfg3 bench each (REPS runs per variant, interleaved):
# the in-tree library ("base") vs cl-rrt_amd/var/<name>/libclrrt.so.  Usage: OUT=<dir> bash tools/ab_bench.sh name...
OUT=${OUT:-abb}
mkdir -p gpurun_out/$OUT
for r in $(seq ${REPS:-2}); do
  for v in base "$@"; do
    if [ $v = base ]; then L=cl-rrt_amd/libclrrt.so; else L=cl-rrt_amd/var/$v/libclrrt.so; fi
    CLRRT_LIB=$L timeout -k 10 150 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-exact --no-sync $BENCH_ARGS \
      > gpurun_out/$OUT/b_${v}_$r.json 2> gpurun_out/$OUT/b_${v}_$r.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/$OUT/b_${v}_$r.json')); print('$v', round(d['value']), round(d['roofline']['avg_launch_ms'],2), {k: round(v) for k,v in d['kernel_ms'].items() if k!='launches'}, d['kernel_ms']['launches']['rollout'])"
  done
done
