#!/bin/bash
# determinism of the two-stream FFT schedule per library variant: tools/split_ab.sh <out> <lib.so>...
set -o pipefail
out=gpurun_out/$1; shift; mkdir -p $out
for L in "$@"; do
  echo "== $L" >> $out/log
  SPLIT_QUICK=1 MP_LIB_PATH=$PWD/$L timeout -k 10 120 python3 tools/split_probe.py fp32_fft 2>&1 | grep -v amdgpu.ids | grep -v alone >> $out/log || exit 1
done
