#!/bin/bash
# fc_1 A/B (repo root): parity tests with each library, fc_1 times per batch for the in-tree library and
# every variant in exp_libs/
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
for lib in "" exp_libs/*.so; do
  echo "== lib ${lib:-in-tree}" >> $out/tests.log
  MP_LIB_PATH=$lib timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -k "pose or fc1 or batch_inv" >> $out/tests.log 2>&1 || exit 1
done
for r in 1 2; do
  for lib in "" exp_libs/*.so; do
    echo "== lib ${lib:-in-tree}" >> $out/fc.log
    MP_LIB_PATH=$lib timeout -k 10 200 python3 tools/time_fc.py --batch 256 128 32 2>&1 | grep -v amdgpu.ids >> $out/fc.log || exit 1
  done
done
