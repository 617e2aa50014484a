#!/bin/bash
# isolated FFT-kernel timings with the inverse kernels' Y reads / P and I writes made wave-contiguous
# (tools/bench_fft.hip built with FFT_PROBE_YCOAL / _PCOAL / _ICOAL: wrong values, same bytes)
set -o pipefail
o=gpurun_out/${1:-ab_fftio}
mkdir -p $o
for rep in 1 2; do
  for n in ${VARIANTS:-base ycoal pcoal both}; do
    timeout -k 10 120 tools/bin/bench_fft_$n 256 5 > $o/bench_fft_${n}_$rep.json 2>> $o/err.log || exit 1
  done
done
