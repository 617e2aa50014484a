#!/bin/bash
# round-5 evidence on one box, into gpurun_out/<tag>/ (copy the summaries into profiles/<tag>/):
#   1. the GPU test suite
#   2. bench.py (fp32, default = the driver's command) and bench.py --dtype bf16
#   3. rocprofv3 kernel-trace stats of the one-stream forward (fp32, bf16) and the PMC byte passes
#      (FETCH_SIZE, WRITE_SIZE: separate runs) -- tools/profile_round.sh
#   4. the PMC byte passes of the DEFAULT (two-stream) fp32 forward
#   5. MFMA-busy PMC pass of the fp32 forward -- tools/pmc_mfma.sh
#   usage (repo root, under gpurun): bash tools/r5_final.sh <tag> [skip-tests]
set -o pipefail
R=$(pwd)
out=$R/gpurun_out/$1
mkdir -p "$out"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$out/gpu_tests.log" 2>&1 || exit 1
fi
timeout -k 10 480 python bench.py > "$out/bench_full_fp32.json" 2> "$out/bench_fp32.err" || exit 1
timeout -k 10 300 python bench.py --dtype bf16 --no-extras > "$out/bench_bf16.json" 2> "$out/bench_bf16.err" || exit 1
bash tools/profile_round.sh "$1" || exit 1
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc "$c" -d "$out/pmc2s_$c" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-extras --no-cpu-baseline --no-parity \
    > "$out/pmc2s_$c.json" 2> "$out/pmc2s_$c.err" || exit 1
done
cd "$R" && bash tools/pmc_mfma.sh "gpurun_out/$1/mfma" || exit 1
echo done > "$out/DONE_FINAL"
