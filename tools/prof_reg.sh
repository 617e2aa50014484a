#!/bin/bash
# rocprofv3 kernel stats of one regressor forward loop (tools/time_regressors.py) -> gpurun_out/<tag>/
# usage (repo root, under gpurun): bash tools/prof_reg.sh <tag> <model> [dtype]
set -eo pipefail
R=$(pwd)
out=$R/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
TR_MODELS=$2 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/kt_$2" -o kt --output-format csv -- \
  python3 "$R/tools/time_regressors.py" 256 ${3:-fp32_split} > "$out/reg_$2_under_rocprof.log" 2> "$out/kt_$2.err"
