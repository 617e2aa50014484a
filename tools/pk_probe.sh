#!/bin/bash
# packed-fp32 FFT determinism + timing per library variant (GPU box, repo root):
#   bash tools/pk_probe.sh <tag> <lib.so>...     -> gpurun_out/<tag>/{det,time}.log
set -o pipefail
dt=${PK_DTYPE:-fp32_fft}
out=gpurun_out/$1; shift; mkdir -p $out
for L in "$@"; do
  echo "== $L" | tee -a $out/det.log >> $out/time.log
  SPLIT_N=256 SPLIT_REPS=5 SPLIT_QUICK=1 MP_LIB_PATH=$PWD/$L timeout -k 10 150 python3 tools/split_probe.py $dt 2>&1 | grep -v amdgpu.ids >> $out/det.log || exit 1
  MP_LIB_PATH=$PWD/$L timeout -k 10 150 python3 tools/time_pose.py --batch 256 --steps 20 --profile --dtype $dt 2>&1 | grep -v amdgpu.ids >> $out/time.log || exit 1
done
