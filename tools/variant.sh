#!/bin/bash
# A/B helper: build/$1/libclrrt.so with extra compile flags ($2) on clrrt_kernels.hip and clrrt_nnwalk.hip
# (the other objects come from the regular in-tree build).  Use with CLRRT_LIB=build/$1/libclrrt.so.
set -e
cd "$(dirname "$0")/../cl-rrt_amd/csrc"
make -s ../libclrrt.so
FLAGS=$(make -s --eval='print-flags: ; @echo $(FLAGS)' print-flags)
out=../../build/$1; mkdir -p $out
/opt/rocm/bin/hipcc $FLAGS $2 -c -o $out/k.o clrrt_kernels.hip &
/opt/rocm/bin/hipcc $FLAGS $2 -c -o $out/w.o clrrt_nnwalk.hip &
wait
/opt/rocm/bin/hipcc $FLAGS -shared -o $out/libclrrt.so $out/k.o $out/w.o clrrt_capi.o
rm -f $out/k.o $out/w.o
