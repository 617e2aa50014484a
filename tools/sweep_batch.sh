#!/bin/bash
# per-batch timing sweep of the hGRU pose forward (GPU box): crops/s at MP_STREAMS=1/2 and the
# single-stream per-kernel profile, for the strong-scaling per-GPU batches 256/128/64/32 (+1, 8)
# usage: bash tools/sweep_batch.sh <outdir> [dtype]
set -eo pipefail
out=$1; dt=${2:-f32_fft}
mkdir -p "$out"
for b in 256 128 64 32 16 8 1; do
  for s in 2 1; do
    MP_STREAMS=$s timeout -k 10 120 python3 tools/time_pose.py --batch $b --dtype $dt --steps 10 \
      $( [ $s = 1 ] && echo --profile ) >> "$out/sweep_$dt.log" 2>&1
  done
done
echo done >> "$out/sweep_$dt.log"
