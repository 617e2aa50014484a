#!/bin/bash
# round-5 first box:
#   1. the four-step loop (k_fft4.hip) against the six-launch loop and the fp64 oracle, timing
#   2. the GPU parity / per-step state tests on it, and the new multi-rank / RCCL tests
#   3. the round-4 state (MP_FFT4=0): default bench, PMC byte passes of the DEFAULT two-stream
#      forward (MP_STREAMS unset), one-stream kernel trace
#   usage (repo root, under gpurun): bash tools/r5_baseline.sh <tag>   -> gpurun_out/<tag>/
set -o pipefail
R=$(pwd)
out=$R/gpurun_out/$1
mkdir -p "$out"
timeout -k 10 300 python tools/fft4_check.py > "$out/fft4_check.log" 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_states.py > "$out/gpu_tests_parity.log" 2>&1
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench_ranks.py \
  > "$out/gpu_tests_ranks.log" 2>&1 || exit 1
export MP_FFT4=0
timeout -k 10 480 python bench.py > "$out/bench_full_fp32_six_launch.json" 2> "$out/bench_fp32.err" || exit 1
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc "$c" -d "$out/pmc2s_$c" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 2 --warmup 1 --no-extras --no-cpu-baseline --no-parity \
    > "$out/pmc2s_$c.json" 2> "$out/pmc2s_$c.err" || exit 1
done
echo done > "$out/DONE"
