#!/bin/bash
# bit identity of the small-batch FFT kernels against the batched ones (tools/fft_det: images [B0, B)
# alone run the latency kernels when B - B0 <= 4)
set -o pipefail
mkdir -p gpurun_out/$1
for a in "6 3" "6 5" "8 4"; do echo "== $a" >> gpurun_out/$1/det.log; timeout -k 10 60 tools/bin/fft_det $a >> gpurun_out/$1/det.log 2>&1 || exit 1; done
