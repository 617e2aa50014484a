#!/bin/bash
# builds tools/bin/fft_stamps_<tag> variants of tools/fft_stamps.hip: usage tools/build_stamps.sh tag "flags" ...
cd "$(dirname "$0")/.."
mkdir -p tools/bin
while [ $# -gt 1 ]; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize $2 -Imonkey-pose_amd/csrc \
    tools/fft_stamps.hip -o tools/bin/fft_stamps_$1 &
  shift 2
done
wait
