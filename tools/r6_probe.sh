#!/bin/bash
# round 6: tests given as args, then PMC passes on the one-stream B = 256 forward (tools/pmc_pass.sh)
#   usage: bash tools/r6_probe.sh <tag> [pytest args...]
set -o pipefail
out=gpurun_out/$1
shift
mkdir -p "$out"
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread "$@" > "$out/gpu_tests.log" 2>&1 || exit 1
fi
for pass in ${PASSES:-tcc ta}; do
  case $pass in
    tcc) C="TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCC_EA0_RDREQ_sum" ;;
    ta) C="TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum" ;;
    bytes) C="FETCH_SIZE" ;;
    wbytes) C="WRITE_SIZE" ;;
    lds) C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY" ;;
    sq) C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" ;;
  esac
  bash tools/pmc_pass.sh "$out" "$pass" ${DT:-f32_fft} -- $C || exit 1
done
echo done > "$out/DONE"
