#!/bin/bash
# A/B of fc_1's 256 x 256 tile (FC_P_BIG, 64 K slices; FC_PB_PIPE fragment reads one group ahead)
# against the 128 x 128 three-block kernel (48 slices): parity tests, fc_1 times per batch (repo root)
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for lib in "" exp_libs/fcpipe0.so exp_libs/fcbig0.so "" exp_libs/fcpipe0.so exp_libs/fcbig0.so; do
  echo "== lib ${lib:-in-tree}" >> $out/fc.log
  MP_LIB_PATH=$lib timeout -k 10 200 python3 tools/time_fc.py --batch 256 192 128 64 32 1 2>&1 | grep -v amdgpu.ids >> $out/fc.log || exit 1
done
