#!/bin/bash
# one box (repo root): batch-1 pose forward time + per-kernel-class HIP-event profile, and the hier
# per-layer profile at B = 256 -> gpurun_out/<tag>/
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
for r in 1 2; do
  timeout -k 10 200 python3 tools/time_pose.py --batch 1 --steps 200 --profile 2>&1 | grep -v amdgpu.ids >> $out/b1.log || exit 1
done
timeout -k 10 200 python3 tools/profile_graph.py hier 256 2>&1 | grep -v amdgpu.ids | head -40 > $out/prof_hier.log || exit 1
timeout -k 10 200 python3 tools/profile_graph.py dense_hier 256 2>&1 | grep -v amdgpu.ids | head -40 > $out/prof_dense_hier.log || exit 1
