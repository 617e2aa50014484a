#!/bin/bash
# A/B of the image order of the B epilogue (MP_EPI_REV) and the spectral GEMM's group passes
# (MP_SPEC_GMAJ): alternating runs of tools/time_pose.py, outputs compared by their printed values
set -o pipefail
o=gpurun_out/${1:-ab_order}
mkdir -p $o
run() {  # rev gmaj streams dtype batch
  MP_EPI_REV=$1 MP_SPEC_GMAJ=$2 MP_STREAMS=$3 timeout -k 10 180 python tools/time_pose.py --dtype $4 --batch $5 --steps 30 \
    2>> $o/err.log | sed "s/^/rev=$1 gmaj=$2 /" | tee -a $o/time.log
}
for rep in 1 2; do
  for cfg in "0 0" "1 0" "0 1" "1 1" "1 2"; do run $cfg 2 f32_fft 256 || exit 1; done
done
for cfg in "0 0" "1 1" "1 2" "0 0" "1 1" "1 2"; do run $cfg 1 f32_fft 256 || exit 1; done
for cfg in "0 0" "1 1" "1 2" "0 0" "1 1" "1 2"; do run $cfg 2 bf16 256 || exit 1; done
for cfg in "0 0" "1 1" "0 0" "1 1"; do run $cfg 2 f32_fft 64 || exit 1; done
