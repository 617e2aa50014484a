#!/bin/bash
# 8-image spectral GEMM with its weights in two halves at 3 blocks per CU (k_fft.hip SPEC_SMALL_HALF)
# A/B: exp_libs/sh0.so (whole-weight registers, 2 blocks per CU) vs sh1.so; parity tests on sh1,
# then alternating small-batch forward timings with the per-kernel HIP-event pass
set -o pipefail
o=gpurun_out/${1:-r4s}
mkdir -p $o
R=$PWD
MP_LIB_PATH=$R/exp_libs/sh1.so timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py > $o/tests.log 2>&1 || exit 1
for r in 1 2; do
  for L in sh0 sh1; do
    for B in 1 8 32; do
      echo "== $L B=$B" >> $o/time.log
      MP_LIB_PATH=$R/exp_libs/$L.so timeout -k 10 200 python3 tools/time_pose.py --batch $B --steps 50 --profile 2>&1 | grep -v amdgpu.ids >> $o/time.log || exit 1
    done
  done
done
