#!/bin/bash
# round-4 GPU checks: the packed-FP32 op_sel probe, the new batch-size parity tests, the bench with
# the in-library HBM probe, and the 2-rank bf16 broadcast rehearsal (gloo, both ranks on one GPU)
set -o pipefail
o=gpurun_out/${1:-r4a}
mkdir -p $o
timeout -k 10 120 tools/bin/pk_hazard > $o/pk_hazard.json 2> $o/pk_hazard.err || exit 1
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py::test_full_size_properties tests/test_gpu_hidden.py > $o/tests.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > $o/bench_full_fp32.json 2> $o/bench_fp32.err || exit 1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --no-extras --dtype bf16 > $o/bench_gloo2_bf16.json 2> $o/bench_gloo2_bf16.err || exit 1
