#!/bin/bash
# Stall breakdown of the pose forward's kernels (one stream, B = 256): one rocprofv3 --pmc pass of up to
# 8 SQ counters (those of the wanted list that `rocprofv3 -L` lists on this box), no tracing beside it.
# usage (GPU box, repo root): bash tools/pmc_stalls.sh <outdir> [dtype]   -> <outdir>/pmc/.../*counter_collection.csv
set -eo pipefail
R=$(pwd)
out=$R/$1
dt=${2:-f32_fft}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$out/avail.txt" 2>&1 || true
WANT="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA"
CTRS=""
for c in $WANT; do grep -qw "$c" "$out/avail.txt" && CTRS="$CTRS $c"; done
echo "counters:$CTRS" > "$out/counters.txt"
MP_STREAMS=1 timeout -s KILL 240 rocprofv3 --pmc $CTRS -d "$out/pmc" -o pmc --output-format csv -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 --no-extras --no-cpu-baseline --no-parity --dtype "$dt" \
  > "$out/pose_$dt.json" 2> "$out/pose_$dt.err"
echo done > "$out/DONE"
