#!/bin/bash
# A/B of the three-blocks-per-CU inverse FFT kernels (FFT_INV3): bit identity of the pose output
# against the two-block build, the parity / states tests, per-kernel times (repo root)
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 120 python3 tools/lib_out.py $out/new.npy 40 > $out/bits.log 2>&1 &&
MP_LIB_PATH=exp_libs/inv3off.so timeout -k 10 120 python3 tools/lib_out.py $out/old.npy 40 >> $out/bits.log 2>&1 &&
python3 -c "import numpy as np; a=np.load('$out/new.npy'); b=np.load('$out/old.npy'); print('bit-identical', np.array_equal(a,b), 'max abs diff', float(np.abs(a-b).max()))" >> $out/bits.log 2>&1 &&
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_states.py -q -x --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for lib in "" exp_libs/inv3off.so "" exp_libs/inv3off.so; do
  echo "== lib ${lib:-in-tree}" >> $out/ab.log
  MP_LIB_PATH=$lib timeout -k 10 200 python3 tools/time_pose.py --batch 256 --steps 20 --profile 2>&1 | grep -v amdgpu.ids >> $out/ab.log || exit 1
done
