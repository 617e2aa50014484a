#!/bin/bash
# one box (repo root): MP_IGEMM_PWN=3 (the one-block pointwise form for 4 cout blocks too) --
# bit-identity, B = 256 regressor tests, whole-model and dense per-layer A/B against 2
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 400 python3 -u -m pytest tests/test_env_variants.py::test_switch_is_bit_identical tests/test_gpu_regressors_b256.py -m gpu -q -x --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for r in 1 2; do
  for f in "2 1" "3 1"; do
    set -- $f; echo "== MP_IGEMM_PWN=$1" >> $out/ab.log
    MP_IGEMM_PWN=$1  timeout -k 10 300 python3 tools/time_regressors.py 256 fp32_split 2>&1 | grep -v amdgpu.ids >> $out/ab.log || exit 1
  done
done
for f in "2 1" "3 1"; do
  set -- $f; echo "== MP_IGEMM_PWN=$1" >> $out/prof_dense.log
  MP_IGEMM_PWN=$1  timeout -k 10 200 python3 tools/profile_graph.py dense 256 2>&1 | grep -v amdgpu.ids | head -30 >> $out/prof_dense.log || exit 1
done


