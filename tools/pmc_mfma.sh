#!/bin/bash
# MFMA-busy and wave-stall PMC pass (rocprofv3, one counter set per run, no tracing beside --pmc)
# over the pose forward (bench.py, one stream: every FFT-path launch is a full-batch launch) and the
# regressors (tools/time_regressors.py): SQ_VALU_MFMA_BUSY_CYCLES with GRBM_GUI_ACTIVE (MfmaUtil =
# busy / (GUI_ACTIVE per XCD x 1024 SIMDs)), and the SQ wait / active split of the wave cycles.
# usage (GPU box, repo root): bash tools/pmc_mfma.sh <outdir> [dtype]    -> parse with tools/pmc_mfma.py
set -eo pipefail
R=$(pwd)
out=$R/$1
dt=${2:-f32_fft}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
CTRS="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
MP_STREAMS=1 timeout -s KILL 240 rocprofv3 --pmc $CTRS -d "$out/pose_$dt" -o pmc --output-format csv -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 --no-extras --no-cpu-baseline --no-parity --dtype "$dt" \
  > "$out/pose_$dt.json" 2> "$out/pose_$dt.err"
timeout -s KILL 240 rocprofv3 --pmc $CTRS -d "$out/regressors" -o pmc --output-format csv -- \
  python3 "$R/tools/time_regressors.py" 256 fp32_split > "$out/regressors.log" 2> "$out/regressors.err"
echo done > "$out/DONE"
