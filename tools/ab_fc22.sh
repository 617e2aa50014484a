#!/bin/bash
# A/B of the 2 x 2 wave fc_1 kernel (k_fc.hip fc_gemm_x3p22_kernel, MP_FC_WL22) on one box
set -o pipefail
o=gpurun_out/fc22
mkdir -p $o
MP_FC_WL22=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "presplit or batch_invariance or pose" -x -q --timeout 120 --timeout-method thread > $o/t.log 2>&1 || exit 1
for v in 0 1 0 1; do MP_FC_WL22=$v timeout -k 10 120 python tools/time_fc.py --batch 256 128 || exit 1; done > $o/fc.log 2>&1 || exit 1
for v in 0 1 0 1; do MP_FC_WL22=$v timeout -k 10 120 python tools/time_pose.py --batch 256 || exit 1; done > $o/pose.log 2>&1 || exit 1
