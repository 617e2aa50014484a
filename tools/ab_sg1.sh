#!/bin/bash
# spectral GEMM one-wave-per-frequency variant at small batches (repo root): MP_SG1_MAX A/B
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
for B in 1 4 8 16 32 64; do
  for v in 0 64; do
    echo "== B=$B MP_SG1_MAX=$v" >> $out/ab.log
    MP_SG1_MAX=$v timeout -k 10 120 python3 tools/time_pose.py --batch $B --steps 30 --profile 2>&1 | grep -v amdgpu.ids >> $out/ab.log || exit 1
  done
done
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -x -k "invariance or split" --timeout 200 --timeout-method thread > $out/tests.log 2>&1
