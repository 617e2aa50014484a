#!/bin/bash
# A/B of the 1x1 sibling fusion (mp_graph.hip) on one box: regressor tests, the env-variant parity
# cases, whole-model timings interleaved, one-stream per-layer profiles of dense.
set -o pipefail
o=gpurun_out/f1x1
mkdir -p $o
timeout -k 10 500 python -u -m pytest tests/test_regressors.py tests/test_dense_hier.py tests/test_env_variants.py -x -q --timeout 200 --timeout-method thread > $o/t.log 2>&1 || exit 1
for v in 0 1 0 1; do MP_GRAPH_FUSE_1X1=$v timeout -k 10 200 python tools/time_regressors.py 256 || exit 1; done > $o/reg.log 2>&1 || exit 1
MP_GRAPH_FUSE_1X1=0 timeout -k 10 200 python tools/profile_graph.py dense 256 > $o/prof_dense0.log 2>&1 || exit 1
MP_GRAPH_FUSE_1X1=1 timeout -k 10 200 python tools/profile_graph.py dense 256 > $o/prof_dense1.log 2>&1 || exit 1
