#!/bin/bash
# one iteration on the box: four-step loop check + timing + per-kernel profile (default, then each
# MP_* A/B setting given in $AB, e.g. AB="MP_FFT4=0"; DT="bf16" adds that dtype's check), then the
# given pytest files
#   usage: [AB="K=V ..."] [DT="bf16"] bash tools/r5_iter.sh <tag> [pytest files...]
set -o pipefail
out=gpurun_out/$1
shift
mkdir -p "$out"
timeout -k 10 300 python tools/fft4_check.py > "$out/fft4_check.log" 2>&1 || exit 1
for dt in $DT; do
  timeout -k 10 300 python tools/fft4_check.py --dtype $dt > "$out/fft4_check_$dt.log" 2>&1 || exit 1
done
for kv in $AB; do   # one A/B setting per word; several variables joined by commas
  env $(echo "$kv" | tr ',' ' ') timeout -k 10 300 python tools/fft4_check.py > "$out/fft4_check_$kv.log" 2>&1 || exit 1
done
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread "$@" > "$out/gpu_tests.log" 2>&1 || exit 1
fi
echo done > "$out/DONE"
