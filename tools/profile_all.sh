#!/bin/bash
# rocprofv3 kernel stats + PMC bytes (profile_round.sh), MFMA busy (pmc_mfma.sh), then the fp32
# bench with extras, on one box.  usage (GPU box, repo root): bash tools/profile_all.sh <tag>
set -o pipefail
bash tools/profile_round.sh "$1" &&
  bash tools/pmc_mfma.sh "gpurun_out/$1/pmc_mfma" f32_fft &&
  timeout -k 10 420 python bench.py > "gpurun_out/$1/bench_full_fp32.json" 2> "gpurun_out/$1/bench_fp32.err"
