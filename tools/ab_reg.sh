#!/bin/bash
# regressor A/B (repo root): regressor GPU tests, then the whole-model times (tools/time_regressors.py)
# and the dense per-layer profile (tools/profile_graph.py) with each env setting given as arguments
# after the tag (e.g. "MP_IGEMM_HALO_NARROW1=0" "MP_IGEMM_HALO_NARROW1=1")
set -o pipefail
out=gpurun_out/$1; shift; mkdir -p $out
timeout -k 10 400 python3 -u -m pytest tests/test_regressors.py tests/test_dense_hier.py tests/test_gpu_regressors_b256.py -m gpu -q -x --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for r in 1 2; do
  for cfg in "$@"; do
    echo "== $cfg" >> $out/ab.log
    env $cfg timeout -k 10 300 python3 tools/time_regressors.py 256 fp32_split 2>&1 | grep -v amdgpu.ids >> $out/ab.log || exit 1
  done
done
for cfg in "$@"; do
  echo "== $cfg" >> $out/prof_dense.log
  env $cfg timeout -k 10 200 python3 tools/profile_graph.py dense 256 2>&1 | grep -v amdgpu.ids | head -30 >> $out/prof_dense.log || exit 1
done
