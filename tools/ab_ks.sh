#!/bin/bash
# fc K-slice length A/B (MP_FC_KSLICE; default rule: ~5,440 -> 48 slices for fc_1): fc_1 alone at
# B = 256 / 64 / 32 / 1 and the whole pose forward at B = 256 / 32, fp32 and bf16
set -o pipefail
o=gpurun_out/ks
mkdir -p $o
for ks in default 2720 1792; do
  e=""; [ $ks != default ] && e="MP_FC_KSLICE=$ks"
  for dt in f32_fft bf16; do
    env $e timeout -k 10 120 python tools/time_fc.py --batch 256 64 32 1 --dtype $dt || exit 1
  done
done > $o/fc.log 2>&1 || exit 1
for ks in default 2720 default 2720; do
  e=""; [ $ks != default ] && e="MP_FC_KSLICE=$ks"
  for B in 256 32; do env $e timeout -k 10 120 python tools/time_pose.py --batch $B || exit 1; done
done > $o/pose.log 2>&1 || exit 1
