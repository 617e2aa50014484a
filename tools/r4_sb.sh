#!/bin/bash
set -o pipefail
o=gpurun_out/r4sb
mkdir -p $o
for r in 1 2; do
  for v in 8 64; do
    for B in 16 32 64; do
      echo "== MP_SPEC_SMALLB=$v B=$B" >> $o/time.log
      MP_SPEC_SMALLB=$v timeout -k 10 200 python3 tools/time_pose.py --batch $B --steps 30 --profile 2>&1 | grep -v amdgpu.ids >> $o/time.log || exit 1
    done
  done
done
