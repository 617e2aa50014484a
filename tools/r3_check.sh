#!/bin/bash
# whole-tree evidence on one box (repo root): the full -m gpu suite, smoke(), the fp32 bench with
# extras and the bf16 bench -> gpurun_out/<tag>/
set -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 &&
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 &&
  timeout -k 10 480 python bench.py > "$out/bench_full_fp32.json" 2> "$out/bench_fp32.err" &&
  timeout -k 10 240 python bench.py --dtype bf16 --no-extras > "$out/bench_bf16.json" 2> "$out/bench_bf16.err"
