# fc_1 variant sweep on one box: <name>:<kslice> pairs, name = base (in-tree) or exp_libs/fc_<name>.so
set -o pipefail
out=gpurun_out/${FCAB_OUT:-fcab3}; mkdir -p $out
for r in 1 2; do
 for v in "$@"; do
  n=${v%%:*}; ks=${v#*:}
  L=""; [ $n != base ] && L=$PWD/exp_libs/fc_$n.so
  echo "== $n ks=$ks r$r" >> $out/ab.log
  MP_LIB_PATH=$L MP_FC_KSLICE=$ks timeout -k 10 120 python3 tools/time_fc.py --dtype f32_fft --batch 256 64 32 2>&1 | grep -v amdgpu.ids >> $out/ab.log || exit 1
 done
done
