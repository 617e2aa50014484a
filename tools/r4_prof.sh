#!/bin/bash
# round-4 rocprofv3 evidence on one box: kernel stats + PMC HBM bytes (tools/profile_round.sh) and
# the MFMA-busy / wave-stall pass (tools/pmc_mfma.sh); summarise with tools/pmc_bytes.py and
# tools/pmc_mfma.py
set -o pipefail
o=gpurun_out/${1:-r4p}
mkdir -p $o
bash tools/profile_round.sh ${1:-r4p} || exit 1
bash tools/pmc_mfma.sh $o/mfma f32_fft || exit 1
