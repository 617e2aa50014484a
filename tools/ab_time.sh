#!/bin/bash
# interleaved same-box timing A/B: for r in 1..$REPS, for each setting in $AB (several variables joined
# by commas; "-" = defaults): tools/time_fwd.py -> gpurun_out/<tag>/times.jsonl
#   usage: AB="- MP_X=1" [REPS=3] [DT=bf16] [BATCH=64] bash tools/ab_time.sh <tag>
set -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
for r in $(seq 1 ${REPS:-3}); do
  for kv in $AB; do
    vars=$( [ "$kv" = "-" ] || echo "$kv" | tr ',' ' ')
    env $vars timeout -k 10 120 python tools/time_fwd.py ${DT:+--dtype $DT} ${BATCH:+--batch $BATCH} >> "$out/times.jsonl" 2> "$out/err.log" || exit 1
  done
done
echo done > "$out/DONE"
