#!/bin/bash
# regressor A/B of library builds (repo root): regressor GPU tests per library, whole-model times and
# the dense per-layer profile for the in-tree library and every variant in exp_libs/
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
for lib in "" exp_libs/*.so; do
  echo "== lib ${lib:-in-tree}" >> $out/tests.log
  MP_LIB_PATH=$lib timeout -k 10 400 python3 -u -m pytest tests/test_regressors.py tests/test_dense_hier.py tests/test_gpu_regressors_b256.py -m gpu -q -x --timeout 200 --timeout-method thread >> $out/tests.log 2>&1 || exit 1
done
for r in 1 2; do
  for lib in "" exp_libs/*.so; do
    echo "== lib ${lib:-in-tree}" >> $out/ab.log
    MP_LIB_PATH=$lib timeout -k 10 300 python3 tools/time_regressors.py 256 fp32_split 2>&1 | grep -v amdgpu.ids >> $out/ab.log || exit 1
  done
done
for lib in "" exp_libs/*.so; do
  echo "== lib ${lib:-in-tree}" >> $out/prof_dense.log
  MP_LIB_PATH=$lib timeout -k 10 200 python3 tools/profile_graph.py dense 256 2>&1 | grep -v amdgpu.ids | head -40 >> $out/prof_dense.log || exit 1
done
