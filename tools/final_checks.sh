#!/bin/bash
# last-session checks on one box: the 2-rank gloo rehearsal of the N > 1 bench path (weak and
# --global-batch strong scaling, both ranks on the one GPU) and the single-GPU bench with extras
set -o pipefail
o=gpurun_out/r2f
mkdir -p $o
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --no-extras > $o/bench_gloo2.json 2> $o/bench_gloo2.err || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 \
  bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --no-extras --global-batch 256 > $o/bench_gloo2_strong.json 2> $o/bench_gloo2_strong.err || exit 1
timeout -k 10 420 python bench.py > $o/bench_full_fp32.json 2> $o/bench_fp32.err || exit 1
