#!/bin/bash
# fc_1 K-loop A/B (repo root): default library vs exp_libs variants (asm reads / asm weight loads / ring depth)
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
for lib in "" exp_libs/fc_asmw0.so exp_libs/fc_asm00.so exp_libs/fc_nst2.so ""; do
  echo "== lib=${lib:-default}" >> $out/fc.log
  MP_LIB_PATH=$lib timeout -k 10 200 python3 tools/time_fc.py --batch 256 128 64 32 8 1 2>&1 | grep -v amdgpu.ids >> $out/fc.log || exit 1
done
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_regressors.py tests/test_gpu_regressors_b256.py -q -x --timeout 200 --timeout-method thread > $out/tests.log 2>&1
