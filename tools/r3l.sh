#!/bin/bash
# fc_1 check + dense / hier per-layer profiles (repo root)
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
bash tools/bisect_fc.sh $1 || exit 1
timeout -k 10 200 python3 tools/profile_graph.py dense 256 > $out/prof_dense.log 2>&1 || exit 1
timeout -k 10 200 python3 tools/profile_graph.py hier 256 > $out/prof_hier.log 2>&1 || exit 1
