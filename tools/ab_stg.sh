#!/bin/bash
# A/B of the staged final B epilogue (k_fft.hip FFT_EPI_STAGE) against exp_libs/stg0.so
set -o pipefail
o=gpurun_out/stg
mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_states.py -x -q --timeout 120 --timeout-method thread > $o/t.log 2>&1 || exit 1
for dt in f32_fft bf16; do
  timeout -k 10 120 python tools/lib_out.py $o/new_$dt.npy 40 $dt && MP_LIB_PATH=$PWD/exp_libs/stg0.so timeout -k 10 120 python tools/lib_out.py $o/old_$dt.npy 40 $dt || exit 1
  python -c "import numpy as np; a=np.load('$o/new_$dt.npy'); b=np.load('$o/old_$dt.npy'); print('$dt bit-identical', np.array_equal(a,b))" >> $o/bitcmp.log 2>&1 || exit 1
done
for i in 1 2; do
  for dt in f32_fft bf16; do
    MP_LIB_PATH=$PWD/exp_libs/stg0.so timeout -k 10 120 python tools/time_pose.py --batch 256 --dtype $dt --profile || exit 1
    timeout -k 10 120 python tools/time_pose.py --batch 256 --dtype $dt --profile || exit 1
  done
done > $o/pose.log 2>&1 || exit 1
