#!/bin/bash
# fc_1 A/B on one box: pre-split LDS-DMA kernel vs the in-loop split (MP_FC_PRESPLIT=0), K slices
# (MP_FC_KSLICE), and variant libraries.  usage: tools/ab_fc.sh <outdir> [name=lib.so ...]
set -o pipefail
out=gpurun_out/$1; shift; mkdir -p $out
for r in 1 2; do
  for ps in ${FC_AB_PRESPLIT:-0 1}; do
    for ks in ${FC_AB_KSLICE:-5440 4096}; do
      for d in f32_fft bf16; do
        echo "== presplit=$ps kslice=$ks $d r$r" >> $out/ab_fc.log
        MP_FC_PRESPLIT=$ps MP_FC_KSLICE=$ks timeout -k 10 120 python3 tools/time_fc.py --dtype $d --batch 256 32 1 2>&1 | grep -v amdgpu.ids >> $out/ab_fc.log || exit 1
      done
    done
  done
  for kv in "$@"; do
    n=${kv%%=*}; L=${kv#*=}
    for d in f32_fft bf16; do
      echo "== $n $d r$r" >> $out/ab_fc.log
      MP_LIB_PATH=$PWD/$L timeout -k 10 120 python3 tools/time_fc.py --dtype $d --batch 256 32 1 2>&1 | grep -v amdgpu.ids >> $out/ab_fc.log || exit 1
    done
  done
done
