# A/B of walk-search builds on one box: the in-tree library vs cl-rrt_amd/var/<name>/libclrrt.so for each
# name given; nn_large at 2.8 and 16 M nodes + a 3-step bench each.  Output: gpurun_out/$OUT
OUT=${OUT:-abw}
mkdir -p gpurun_out/$OUT
for v in base "$@"; do
  if [ $v = base ]; then L=cl-rrt_amd/libclrrt.so; else L=cl-rrt_amd/var/$v/libclrrt.so; fi
  CLRRT_LIB=$L timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-exact > gpurun_out/$OUT/b_$v.json 2> gpurun_out/$OUT/b_$v.err || exit 1
  CLRRT_LIB=$L timeout -k 10 250 python3 -u tools/nn_large.py ${SIZES:-2.8 16} > gpurun_out/$OUT/nn_$v.txt 2>&1 || exit 1
done
