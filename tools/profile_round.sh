#!/bin/bash
# rocprofv3 evidence for one profiles/<tag> directory, on the GPU box:
#   1. kernel-trace stats of the single-stream bench (MP_STREAMS=1: every FFT-path launch is a whole
#      256-crop batch, as in bench.py's HIP-event roofline pass), fp32 FFT path and bf16;
#   2. the two PMC passes (FETCH_SIZE, WRITE_SIZE -- separate runs) per dtype, combined later by
#      tools/pmc_bytes.py with the gfx950 FETCH_SIZE x2 correction (MI355X_MICROARCH.md).
# usage (from the repo root, under gpurun): bash tools/profile_round.sh <tag>   -> gpurun_out/<tag>/
set -eo pipefail
R=$(pwd)
out=$R/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for d in f32_fft bf16; do
  MP_STREAMS=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/kt_$d" -o kt --output-format csv -- \
    python3 "$R/bench.py" --steps 5 --warmup 1 --no-extras --no-cpu-baseline --dtype "$d" \
    > "$out/bench_${d}_1stream_under_rocprof.json" 2> "$out/kt_$d.err"
  for c in FETCH_SIZE WRITE_SIZE; do
    MP_STREAMS=1 timeout -s KILL 180 rocprofv3 --pmc "$c" -d "$out/pmc_${d}_$c" -o pmc --output-format csv -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 --no-extras --no-cpu-baseline --no-parity --dtype "$d" \
      > "$out/pmc_${d}_$c.json" 2> "$out/pmc_${d}_$c.err"
  done
done
echo done > "$out/DONE"
