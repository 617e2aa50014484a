#!/bin/bash
# per-batch env A/B: lines "BATCH setting setting ..." in $SWEEP (';'-separated)
#   SWEEP="256 - MP_STREAMS=3;64 - MP_STREAMS=1" bash tools/r6_envsweep.sh <tag>
set -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
IFS=';' read -ra lines <<< "$SWEEP"
for ln in "${lines[@]}"; do
  set -- $ln
  b=$1; shift
  timeout -k 10 600 python -u tools/ab_env.py --reps ${REPS:-2} --batch $b --dtype ${DT:-f32_fft} "$@" >> "$out/ab.jsonl" 2>> "$out/ab.err" || exit 1
done
echo done > "$out/DONE"
