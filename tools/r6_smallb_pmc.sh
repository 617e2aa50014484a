#!/bin/bash
# PMC HBM bytes per pose forward at small batches (default schedule), for the bytes-floor account of the
# strong-scaling rows: FETCH_SIZE and WRITE_SIZE passes of bench.py --batch B (tools/pmc_forward_raw.py)
#   usage (repo root, under gpurun): bash tools/r6_smallb_pmc.sh <tag> [batches...]
set -o pipefail
R=$(pwd)
out=$R/gpurun_out/$1
shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for b in "${@:-32 64}"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc "$c" -d "$out/b${b}_$c" -o pmc --output-format csv -- \
      python3 "$R/bench.py" --batch "$b" --steps 3 --warmup 1 --no-extras --no-cpu-baseline --no-parity \
      > "$out/b${b}_$c.json" 2> "$out/b${b}_$c.err" || exit 1
  done
done
echo done > "$out/DONE"
