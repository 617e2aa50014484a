#!/bin/bash
# FFT kernels with and without their transforms (data movement alone), and per-launch kernel traces
# of the batch-1 / batch-32 forward (does the Infinity Cache serve the 87 MB of spectral weights?)
set -o pipefail
o=gpurun_out/${1:-r4b}
mkdir -p $o
timeout -k 10 120 tools/bin/bench_fft 256 5 > $o/bench_fft.json 2> $o/bench_fft.err || exit 1
timeout -k 10 120 tools/bin/bench_fft_nofft 256 5 > $o/bench_fft_nofft.json 2> $o/bench_fft_nofft.err || exit 1
for b in 1 32; do
  timeout -k 10 240 rocprofv3 --kernel-trace -d $o/kt_b$b -o kt --output-format csv -- \
    python3 tools/time_pose.py --batch $b --steps 5 > $o/time_b$b.log 2>&1 || exit 1
done
