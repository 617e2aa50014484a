#!/bin/bash
# regressor A/B (repo root): default library vs exp_libs/igemm_old.so; then the regressor GPU tests
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
for lib in "" exp_libs/igemm_old.so "" exp_libs/igemm_old.so; do
  echo "== lib=${lib:-default}" >> $out/reg.log
  MP_LIB_PATH=$lib timeout -k 10 300 python3 tools/time_regressors.py 256 fp32_split bf16 2>&1 | grep -v amdgpu.ids >> $out/reg.log || exit 1
done
timeout -k 10 600 python3 -u -m pytest tests/test_regressors.py tests/test_gpu_regressors_b256.py tests/test_dense_hier.py tests/test_attn.py -q -x --timeout 300 --timeout-method thread > $out/tests.log 2>&1
