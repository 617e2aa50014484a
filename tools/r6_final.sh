#!/bin/bash
# round-6 evidence on one box, into gpurun_out/<tag>/ (summaries then copied into profiles/r6/ with
# the tree's STAMP.json).  Two parts, one GPU call each:
#   part A: the GPU test suite; bench.py (fp32 = the driver's command, with the bf16 extras leg)
#   part B: rocprofv3 kernel-trace stats of the one-stream forward (fp32, bf16) and the PMC byte passes
#           (tools/profile_round.sh); the PMC byte passes of the default (two-stream) fp32 forward; the
#           MFMA-busy / stall pass (tools/pmc_mfma.sh)
#   usage (repo root, under gpurun): bash tools/r6_final.sh <tag> A|B
set -o pipefail
R=$(pwd)
out=$R/gpurun_out/$1
mkdir -p "$out"
cp -f "$R/profiles/TREE_STAMP.json" "$out/STAMP_$2.json" 2>/dev/null
if [ "$2" = A ]; then
  timeout -k 10 780 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$out/gpu_tests.log" 2>&1 || exit 1
  timeout -k 10 400 python bench.py > "$out/bench_full_fp32.json" 2> "$out/bench_fp32.err" || exit 1
  echo done > "$out/DONE_A"
else
  bash tools/profile_round.sh "$1" || exit 1
  cd /tmp && export TMPDIR=/tmp
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc "$c" -d "$out/pmc2s_$c" -o pmc --output-format csv -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 --no-extras --no-cpu-baseline --no-parity \
      > "$out/pmc2s_$c.json" 2> "$out/pmc2s_$c.err" || exit 1
  done
  cd "$R" && bash tools/pmc_mfma.sh "gpurun_out/$1/mfma" || exit 1
  echo done > "$out/DONE_B"
fi
