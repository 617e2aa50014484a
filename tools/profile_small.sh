#!/bin/bash
# rocprofv3 kernel-trace stats of the one-stream fp32 forward at the small per-GPU batches of the
# strong-scaling reading (B = 32: 8 GPUs x 32 = 256) and at batch 1 (config 5)
set -eo pipefail
R=$(pwd)
out=$R/gpurun_out/$1
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for B in 32 1; do
  MP_STREAMS=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/kt_b$B" -o kt --output-format csv -- \
    python3 "$R/bench.py" --batch $B --steps 10 --warmup 2 --no-extras --no-cpu-baseline --no-parity \
    > "$out/bench_b${B}_1stream_under_rocprof.json" 2> "$out/kt_b$B.err"
done
echo done > "$out/DONE"
