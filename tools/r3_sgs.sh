#!/bin/bash
# one box (repo root): MP_SPEC_SMALLB (8-image spectral GEMM tiles up to batch N) -- bit-identity,
# parity / state tests with it at 64, forward times at B = 16 / 32 / 64 with 8 / 32 / 64
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 300 python3 -u -m pytest "tests/test_env_variants.py::test_switch_is_bit_identical" -m gpu -q -x --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
MP_SPEC_SMALLB=64 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_states.py -m gpu -q -x --timeout 200 --timeout-method thread >> $out/tests.log 2>&1 || exit 1
for r in 1 2; do
  for b in 16 32 64; do
    for v in 8 32 64; do
      echo "== MP_SPEC_SMALLB=$v B=$b" >> $out/ab.log
      MP_SPEC_SMALLB=$v timeout -k 10 200 python3 tools/time_pose.py --batch $b --steps 50 2>&1 | grep -v amdgpu.ids >> $out/ab.log || exit 1
    done
  done
done
