#!/bin/bash
# the small-batch FFT kernels after a change (repo root): bit identity against the batched kernels,
# parity / states tests, phase stamps and forward times at B = 1, 4, 8
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 60 tools/bin/lfft_diff > $out/diff.log 2>&1 &&
for a in "6 3" "12 4"; do echo "== $a" >> $out/det.log; timeout -k 10 60 tools/bin/fft_det $a >> $out/det.log 2>&1 || exit 1; done &&
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_states.py -q -x --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for b in 1 8; do echo "== B=$b" >> $out/stamps.log; timeout -k 10 60 tools/bin/fft_stamps $b >> $out/stamps.log 2>&1 || exit 1; done
for b in 1 4 8; do
  echo "== B=$b" >> $out/ab.log
  timeout -k 10 200 python3 tools/time_pose.py --batch $b --steps 50 --profile 2>&1 | grep -v amdgpu.ids >> $out/ab.log || exit 1
done
