#!/bin/bash
# round-4 full GPU check on one box: the -m gpu suite, smoke, and the default bench (extras included)
set -o pipefail
o=gpurun_out/${1:-r4e}
mkdir -p $o
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $o/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 900 python bench.py > $o/bench_full_fp32.json 2> $o/bench_fp32.err || exit 1
