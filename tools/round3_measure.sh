#!/bin/bash
# milestone evidence on one box (repo root): new GPU tests, smoke(), the full fp32 bench with extras,
# the bf16 bench -> gpurun_out/<tag>/
set -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
timeout -k 10 300 python -u -m pytest tests/test_crop_reference.py tests/test_gpu_hidden.py -m gpu -q --timeout 200 --timeout-method thread > "$out/gpu_tests_new.log" 2>&1 &&
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 &&
  timeout -k 10 480 python bench.py > "$out/bench_full_fp32.json" 2> "$out/bench_fp32.err" &&
  timeout -k 10 240 python bench.py --dtype bf16 --no-extras > "$out/bench_bf16.json" 2> "$out/bench_bf16.err"
