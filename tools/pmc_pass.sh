#!/bin/bash
# one rocprofv3 --pmc pass (no tracing beside it) over a short one-stream B = 256 pose forward:
#   usage (GPU box, repo root): bash tools/pmc_pass.sh <outdir> <tag> [dtype] -- <counters...>
# -> <outdir>/<tag>/pmc/.../*counter_collection.csv, <outdir>/<tag>/head.txt (the git head of the tree)
set -eo pipefail
R=$(pwd)
base=$R/$1
out=$base/$2
dt=${3:-f32_fft}
shift 3
[ "$1" = "--" ] && shift
mkdir -p "$out"
cp -f "$R/profiles/TREE_STAMP.json" "$out/STAMP.json" 2>/dev/null || true
cd /tmp && export TMPDIR=/tmp
[ -s "$base/avail.txt" ] || timeout -s KILL 60 rocprofv3 -L > "$base/avail.txt" 2>&1 || true
CTRS=""
for c in "$@"; do grep -qw "${c%_sum}" "$base/avail.txt" && CTRS="$CTRS $c"; done
echo "counters:$CTRS (asked: $*)" > "$out/counters.txt"
[ -n "$CTRS" ] || exit 3
MP_STREAMS=1 timeout -s KILL 120 rocprofv3 --pmc $CTRS -d "$out/pmc" -o pmc --output-format csv -- \
  python3 "$R/bench.py" --steps 2 --warmup 1 --no-extras --no-cpu-baseline --no-parity --dtype "$dt" \
  > "$out/pose_$dt.json" 2> "$out/pose_$dt.err"
echo done > "$out/DONE"
