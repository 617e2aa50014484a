#!/bin/bash
# A/B of library variants on one box: tools/ab_run.sh <outdir> <name>=<lib.so> ... (new = the in-tree lib)
# each variant: tools/time_pose.py --profile, fp32 and bf16, two alternating rounds
set -o pipefail
out=gpurun_out/$1; shift; mkdir -p $out
for r in 1 2; do
  for kv in "$@"; do
    n=${kv%%=*}; L=${kv#*=}
    for d in f32_fft bf16; do
      echo "== $n $d r$r" >> $out/ab.log
      MP_LIB_PATH=$PWD/$L timeout -k 10 120 python3 tools/time_pose.py --dtype $d --profile 2>&1 | grep -v amdgpu.ids >> $out/ab.log || exit 1
    done
  done
done
