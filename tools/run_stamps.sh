#!/bin/bash
# runs every tools/bin/fft_stamps_* variant (fp32 and bf16, two rounds) -> gpurun_out/$1/stamps.log
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
for r in 1 2; do
  for v in tools/bin/fft_stamps_*; do
    for d in f32 bf16; do
      echo "== $(basename $v) $d round $r" >> $out/stamps.log
      timeout -k 10 60 $v 256 $d >> $out/stamps.log 2>&1 || exit 1
    done
  done
done
