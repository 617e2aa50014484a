#!/bin/bash
# rocprofv3 kernel stats + PMC bytes of single convs (tools/conv_bench.py) -> gpurun_out/<tag>/
# usage (repo root, under gpurun): bash tools/prof_conv.sh <tag> <shape> ...
set -eo pipefail
R=$(pwd)
out=$R/gpurun_out/$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/kt" -o kt --output-format csv -- \
  python3 "$R/tools/conv_bench.py" 256 "$@" > "$out/conv_under_rocprof.log" 2> "$out/kt.err"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc "$c" -d "$out/pmc_$c" -o pmc --output-format csv -- \
    python3 "$R/tools/conv_bench.py" 256 "$@" > "$out/pmc_$c.log" 2> "$out/pmc_$c.err"
done
echo done > "$out/DONE"
