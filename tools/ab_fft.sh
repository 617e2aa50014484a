#!/bin/bash
# FFT-kernel variant A/B on one box (repo root): tools/ab_fft.sh <tag> <lib.so>...  (time_pose --profile per library)
set -o pipefail
out=gpurun_out/$1; shift; mkdir -p $out
for L in "$@"; do
  echo "== $L" >> $out/ab.log
  MP_LIB_PATH=$PWD/$L timeout -k 10 200 python3 tools/time_pose.py --batch 256 --steps 20 --profile 2>&1 | grep -v amdgpu.ids >> $out/ab.log || exit 1
done
