#!/bin/bash
# A/B of the 8-image spectral GEMM for batches <= 8 (spec_gemm_kernel<0, 8>, SPEC_SMALLB): parity /
# states tests, forward times at B = 1 .. 8 with it (3 and 2 blocks per CU) and without (repo root)
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_states.py -q -x --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for b in 1 4 8; do
  for lib in "" exp_libs/sg_minb2.so exp_libs/sg_off.so; do
    echo "== lib ${lib:-in-tree} B=$b" >> $out/ab.log
    MP_LIB_PATH=$lib timeout -k 10 200 python3 tools/time_pose.py --batch $b --steps 50 --profile 2>&1 | grep -v amdgpu.ids >> $out/ab.log || exit 1
  done
done
