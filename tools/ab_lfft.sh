#!/bin/bash
# A/B of the small-batch 9-lane FFT kernels (k_fft.hip lfft_*): bit identity against the batched
# kernels (tools/fft_det, tools/lfft_diff), parity / states tests, then the forward at B = 1 .. 16
# with them off (MP_LFFT_MAXB=0) and on for every batch (=16), and B = 256 against the previous
# k_fft.hip (exp_libs/fft_head.so) (repo root)
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 60 tools/bin/lfft_diff > $out/diff.log 2>&1 &&
for a in "6 3" "6 5"; do echo "== $a" >> $out/det.log; timeout -k 10 60 tools/bin/fft_det $a >> $out/det.log 2>&1 || exit 1; done &&
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_states.py -q -x --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for b in 1 2 4 8 16; do
  for mb in 0 16; do
    echo "== MP_LFFT_MAXB=$mb B=$b" >> $out/ab.log
    MP_LFFT_MAXB=$mb timeout -k 10 200 python3 tools/time_pose.py --batch $b --steps 50 --profile 2>&1 | grep -v amdgpu.ids >> $out/ab.log || exit 1
  done
done
for lib in ""; do
  echo "== lib ${lib:-in-tree} B=256" >> $out/ab.log
  MP_LIB_PATH=$lib timeout -k 10 200 python3 tools/time_pose.py --batch 256 --steps 20 --profile 2>&1 | grep -v amdgpu.ids >> $out/ab.log || exit 1
done
