#!/bin/bash
# round-3 A/B on one box (repo root): fc_1 ring kernel (MP_FC_RING, old slicing MP_FC_KSLICE=5440) and
# the double-buffered backbone halo (MP_CONV_DB); per-kernel HIP-event times + whole-forward time
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_states.py -q -x --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
for cfg in "MP_FC_RING=0 MP_FC_KSLICE=5440 MP_CONV_DB=0" "MP_FC_RING=1" "MP_FC_RING=0" "MP_CONV_DB=0" "MP_FC_RING=0 MP_FC_KSLICE=5440 MP_CONV_DB=0" "MP_FC_RING=1"; do
  echo "== $cfg" >> $out/ab.log
  env $cfg timeout -k 10 200 python3 tools/time_pose.py --batch 256 --steps 20 --profile 2>&1 | grep -v amdgpu.ids >> $out/ab.log || exit 1
done
for cfg in "MP_FC_RING=0 MP_FC_KSLICE=5440 MP_CONV_DB=0" "MP_FC_RING=1"; do
  echo "== $cfg" >> $out/fc.log
  env $cfg timeout -k 10 200 python3 tools/time_fc.py --batch 256 192 128 64 32 1 2>&1 | grep -v amdgpu.ids >> $out/fc.log || exit 1
done
