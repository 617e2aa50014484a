#!/bin/bash
# round-4 evidence on one box: hipGraph concurrency and spectrum-layout probes, then rocprofv3
# kernel stats + PMC HBM bytes (tools/profile_round.sh) and the MFMA-busy pass (tools/pmc_mfma.sh)
set -o pipefail
o=gpurun_out/${1:-r4p}
mkdir -p $o
timeout -k 10 60 tools/bin/graph_concurrency > $o/graph_concurrency.json 2> $o/graph_concurrency.err || exit 1
timeout -k 10 120 tools/bin/spec_layout_probe > $o/spec_layout_probe.json 2> $o/spec_layout_probe.err || exit 1
bash tools/profile_round.sh ${1:-r4p} || exit 1
bash tools/pmc_mfma.sh $o/mfma f32_fft || exit 1
