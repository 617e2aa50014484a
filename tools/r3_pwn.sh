#!/bin/bash
# one box (repo root): the new GPU tests, the MP_IGEMM_PWN A/B of the regressors (whole models twice,
# dense per-layer profile), then rocprofv3 kernel stats + PMC bytes + MFMA busy of the pose forward
# -> gpurun_out/<tag>/
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_stream_pipeline.py tests/test_env_variants.py tests/test_regressors.py tests/test_gpu_regressors_b256.py -m gpu -q -x --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for r in 1 2; do
  for f in 1 0 2; do
    echo "== MP_IGEMM_PWN=$f" >> $out/ab.log
    MP_IGEMM_PWN=$f timeout -k 10 300 python3 tools/time_regressors.py 256 fp32_split 2>&1 | grep -v amdgpu.ids >> $out/ab.log || exit 1
  done
done
for f in 1 0 2; do
  echo "== MP_IGEMM_PWN=$f" >> $out/prof_dense.log
  MP_IGEMM_PWN=$f timeout -k 10 200 python3 tools/profile_graph.py dense 256 2>&1 | grep -v amdgpu.ids | head -30 >> $out/prof_dense.log || exit 1
done
bash tools/profile_round.sh $1/prof || exit 1
bash tools/pmc_mfma.sh gpurun_out/$1/mfma || exit 1
