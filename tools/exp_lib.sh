#!/bin/bash
# build an A/B variant of libmonkeypose.so: one source recompiled with extra flags, linked with the
# in-tree objects.  usage: tools/exp_lib.sh <source.hip> <out.so> <flags...>   (load it with MP_LIB_PATH;
# a source outside csrc/, e.g. an older revision: EXP_BASE=<name of the object it replaces>)
set -e
cd "$(dirname "$0")/../monkey-pose_amd/csrc"
src=$1; out=$2; shift 2
obj=/tmp/exp_$(basename "$out" .so).o
# the Makefile's per-source flags (k_fft.hip: -fno-slp-vectorize -- without it the FFT kernels are
# SLP-packed, spill, and round differently)
extra=""; [ "$(basename "$src")" = k_fft.hip ] && extra="-fno-slp-vectorize"
[ "$(basename "$src")" = k_fft4.hip ] && extra="-fno-slp-vectorize -ffp-contract=on"
/opt/rocm/bin/hipcc $extra --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result "$@" -c "$src" -o "$obj"
base=${EXP_BASE:-$(basename "${src%.hip}")}   # the in-tree object the variant replaces (EXP_BASE for a copy elsewhere)
objs=$(ls build/*.o | grep -v "build/${base}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out" $objs "$obj" -Wl,-rpath,/opt/rocm/lib
