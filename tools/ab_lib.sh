#!/bin/bash
# same-box A/B of the in-tree library against variant builds (tools/exp_lib.sh -> exp_libs/<name>.so):
# alternating tools/time_pose.py runs (with its one-stream per-kernel profile).
# usage: tools/ab_lib.sh <out> "<variant.so> ..." "<dtype batch>"...
set -o pipefail
o=gpurun_out/$1; libs=$2; shift 2
mkdir -p $o
for cfg in "$@"; do
  set -- $cfg
  for rep in 1 2; do
    for L in tree $libs; do
      if [ $L = tree ]; then unset MP_LIB_PATH; else export MP_LIB_PATH=$L; fi
      timeout -k 10 180 python tools/time_pose.py --dtype $1 --batch $2 --steps 30 --profile 2>> $o/err.log \
        | sed "s|^|lib=$L |" | tee -a $o/time.log || exit 1
    done
  done
done
