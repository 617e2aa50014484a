#!/bin/bash
# A/B of the backbone tile rows (k_conv64x3.hip conv_tile_rows; MP_CONV_TH forces 8 / 16 / 32)
set -o pipefail
o=gpurun_out/th2
mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "small_batch_tiles or batch_invariance" -x -q --timeout 160 --timeout-method thread > $o/t.log 2>&1 || exit 1
for B in 32 24; do
  for th in 8 16 32 8 16 32; do MP_CONV_TH=$th timeout -k 10 120 python tools/time_pose.py --batch $B --profile || exit 1; done
done > $o/pose.log 2>&1 || exit 1
