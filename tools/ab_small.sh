#!/bin/bash
# small-batch A/B (repo root): parity / states tests, then forward times at B = 1, 4, 8 for the
# in-tree library and the variants in exp_libs/ (one line per library and batch)
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_states.py -q -x --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for b in 1 4 8; do
  for lib in "" exp_libs/*.so; do
    echo "== lib ${lib:-in-tree} B=$b" >> $out/ab.log
    MP_LIB_PATH=$lib timeout -k 10 200 python3 tools/time_pose.py --batch $b --steps 50 --profile 2>&1 | grep -v amdgpu.ids >> $out/ab.log || exit 1
  done
done
