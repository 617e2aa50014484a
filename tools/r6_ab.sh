#!/bin/bash
# round 6 iteration on the box: pytest args (optional, before "--"), then tools/ab_env.py settings
#   usage: [REPS=2] [BATCH=256] [DT=f32_fft] bash tools/r6_ab.sh <tag> [pytest args...] -- <settings...>
set -o pipefail
out=gpurun_out/$1
shift
mkdir -p "$out"
tests=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do tests+=("$1"); shift; done
[ "$1" = "--" ] && shift
if [ ${#tests[@]} -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread "${tests[@]}" > "$out/gpu_tests.log" 2>&1 || exit 1
fi
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u tools/ab_env.py --reps ${REPS:-2} --batch ${BATCH:-256} --dtype ${DT:-f32_fft} "$@" > "$out/ab.jsonl" 2> "$out/ab.err" || exit 1
fi
echo done > "$out/DONE"
