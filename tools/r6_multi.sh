#!/bin/bash
# several steps in one GPU call, each bounded, stopping at the first failure:
#   AB="<settings>" PASSES="<pmc passes>" TESTS="<pytest args>" bash tools/r6_multi.sh <tag>
set -o pipefail
tag=$1
mkdir -p gpurun_out/$tag
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread $TESTS > gpurun_out/$tag/gpu_tests.log 2>&1 || exit 1
fi
if [ -n "$AB" ]; then
  timeout -k 10 900 python -u tools/ab_env.py --reps ${REPS:-2} --batch ${BATCH:-256} --dtype ${DT:-f32_fft} $AB > gpurun_out/$tag/ab.jsonl 2> gpurun_out/$tag/ab.err || exit 1
fi
if [ -n "$PASSES" ]; then
  PASSES="$PASSES" bash tools/r6_probe.sh $tag || exit 1
fi
echo done > gpurun_out/$tag/DONE
