#!/bin/bash
# ab_env.py at several batches: BATCHES="128 64 32" AB="<settings>" bash tools/r6_sweep.sh <tag>
set -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
for b in ${BATCHES:-128 64 32}; do
  timeout -k 10 600 python -u tools/ab_env.py --reps ${REPS:-2} --batch $b --dtype ${DT:-f32_fft} $AB >> "$out/ab.jsonl" 2>> "$out/ab.err" || exit 1
done
echo done > "$out/DONE"
