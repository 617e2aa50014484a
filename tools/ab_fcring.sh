#!/bin/bash
# fc_1 ring kernel A/B on one box (repo root): the old form = MP_FC_RING=0 MP_FC_KSLICE=5440 (48 slices)
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
for cfg in "MP_FC_RING=0 MP_FC_KSLICE=5440" "MP_FC_RING=0" "MP_FC_RING=1" "MP_FC_RING=0 MP_FC_KSLICE=5440" "MP_FC_RING=1"; do
  echo "== $cfg" >> $out/fc.log
  env $cfg timeout -k 10 200 python3 tools/time_fc.py --batch 256 128 64 32 1 2>&1 | grep -v amdgpu.ids >> $out/fc.log || exit 1
  env $cfg timeout -k 10 200 python3 tools/time_pose.py --batch 256 --steps 20 2>&1 | grep -v amdgpu.ids >> $out/fc.log || exit 1
done
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1
