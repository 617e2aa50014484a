#!/bin/bash
# same-box A/B on the box: tools/fft4_check.py under each setting in $AB (one per word, several
# variables joined by commas; "-" = defaults), then, for each setting in $PMC, the two PMC byte passes
# (FETCH_SIZE, WRITE_SIZE) of the default two-stream bench forward -> gpurun_out/<tag>/
#   usage: AB="- MP_X=0" [PMC="- MP_X=0"] [DT=bf16] bash tools/r5_ab.sh <tag>
set -o pipefail
R=$(pwd)
out=$R/gpurun_out/$1
mkdir -p "$out"
i=0
for kv in $AB; do   # (a setting may repeat: interleaved repeats, logs numbered in run order)
  i=$((i + 1))
  vars=$( [ "$kv" = "-" ] || echo "$kv" | tr ',' ' ')
  env $vars timeout -k 10 300 python tools/fft4_check.py ${DT:+--dtype $DT} ${QUICK:+--quick} > "$out/ab_${i}_$kv.log" 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for kv in $PMC; do
  vars=$( [ "$kv" = "-" ] || echo "$kv" | tr ',' ' ')
  for c in FETCH_SIZE WRITE_SIZE; do
    env $vars timeout -s KILL 180 rocprofv3 --pmc "$c" -d "$out/pmc_${kv}_$c" -o pmc --output-format csv -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 --no-extras --no-cpu-baseline --no-parity \
      > "$out/pmc_${kv}_$c.json" 2> "$out/pmc_${kv}_$c.err" || exit 1
  done
done
echo done > "$out/DONE"
