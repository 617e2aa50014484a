#!/bin/bash
# fc_1 final form check + dense pointwise conv probes (repo root)
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/time_fc.py --batch 256 64 1 2>&1 | grep -v amdgpu.ids > $out/fc.log || exit 1
S="64,64,184,64,1 64,64,120,48,1 64,64,72,32,1 64,64,40,24,1 32,32,496,128,1 32,32,304,96,1 64,64,184,96,1 64,64,64,96,3 64,64,24,32,3 64,64,16,24,3 64,64,64,96,3,2"
for pw in 1 0; do
  echo "== MP_IGEMM_PW=$pw" >> $out/conv.log
  MP_IGEMM_PW=$pw timeout -k 10 200 python3 tools/conv_bench.py 256 $S 2>&1 | grep -v amdgpu.ids >> $out/conv.log || exit 1
done
