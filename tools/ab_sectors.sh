mkdir -p gpurun_out/r04l
for v in base ap16 ap32; do
  if [ $v = base ]; then L=cl-rrt_amd/libclrrt.so; else L=cl-rrt_amd/var/$v/libclrrt.so; fi
  CLRRT_LIB=$L timeout -k 10 250 python3 -u tools/nn_large.py 2.8 5.5 16 > gpurun_out/r04l/nn_$v.txt 2>&1 || exit 1
  CLRRT_LIB=$L timeout -k 10 200 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-exact > gpurun_out/r04l/b_$v.json 2> gpurun_out/r04l/b_$v.err || exit 1
done
