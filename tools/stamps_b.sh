set -o pipefail
mkdir -p gpurun_out/r3u
for b in 1 4 32 256; do echo "== B=$b" >> gpurun_out/r3u/stamps.log; timeout -k 10 60 tools/bin/fft_stamps $b >> gpurun_out/r3u/stamps.log 2>&1 || exit 1; done
