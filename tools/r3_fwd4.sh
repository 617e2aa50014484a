#!/bin/bash
# one box (repo root): MP_FFT_FWD4 (fp32 forward FFT at 4 blocks per CU) -- bit-identity and the pose
# GPU tests with it on, the fp32 bench alternating off / on, rocprofv3 kernel stats of both (one
# stream) -> gpurun_out/<tag>/
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
R=$(pwd)
timeout -k 10 300 python3 -u -m pytest "tests/test_env_variants.py::test_switch_is_bit_identical" -m gpu -q -x --timeout 200 --timeout-method thread > $out/tests.log 2>&1 || exit 1
MP_FFT_FWD4=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_states.py -m gpu -q -x --timeout 200 --timeout-method thread >> $out/tests.log 2>&1 || exit 1
for r in 1 2 3; do
  for f in 0 1; do
    echo "== MP_FFT_FWD4=$f" >> $out/ab.log
    MP_FFT_FWD4=$f timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline --no-parity 2>/dev/null >> $out/ab.log || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for f in 0 1; do
  MP_FFT_FWD4=$f MP_STREAMS=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/$out/kt_$f" -o kt --output-format csv -- \
    python3 "$R/bench.py" --steps 5 --warmup 1 --no-extras --no-cpu-baseline --no-parity > "$R/$out/kt_$f.json" 2> "$R/$out/kt_$f.err" || exit 1
done
