#!/bin/bash
# End-of-milestone GPU evidence on one box: the -m gpu suite, smoke(), the fp32 bench with extras and
# the bf16 bench -> gpurun_out/<tag>/.  Profiles: tools/profile_round.sh and tools/pmc_mfma.sh.
# usage (GPU box, repo root): bash tools/round_measure.sh <tag>
set -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$out/gpu_tests.log" 2>&1 &&
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 &&
  timeout -k 10 420 python bench.py > "$out/bench_full_fp32.json" 2> "$out/bench_fp32.err" &&
  timeout -k 10 240 python bench.py --dtype bf16 --no-extras > "$out/bench_bf16.json" 2> "$out/bench_bf16.err"
