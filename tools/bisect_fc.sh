#!/bin/bash
# fc_1 K-loop variants: correctness (golden / planes / batch invariance) and timing (repo root)
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
for lib in "" exp_libs/fc_asmw0.so; do
  echo "== lib=${lib:-default}" >> $out/bisect.log
  MP_LIB_PATH=$lib timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q --timeout 200 --timeout-method thread 2>&1 | grep -E "passed|failed|Error:" >> $out/bisect.log
  MP_LIB_PATH=$lib timeout -k 10 200 python3 tools/time_fc.py --batch 256 64 1 2>&1 | grep -v amdgpu.ids >> $out/bisect.log || exit 1
done
exit 0
