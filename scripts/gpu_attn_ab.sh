#!/bin/bash
# Interleaved A/B of two attention builds: old = ab_lib/libtdl_kernels_old.so (the experiment's
# build, env EXP_ENV applied), new = in-tree (3 rounds)
mkdir -p gpurun_out
out=gpurun_out/attn_ab.txt
: > $out
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then
      line=$(env TDL_NATIVE_LIB=$PWD/ab_lib/libtdl_kernels_old.so ${EXP_ENV} timeout -k 10 120 python -u scripts/attn_time.py 2>/dev/null | grep '^{') || exit 1
    else
      line=$(timeout -k 10 120 python -u scripts/attn_time.py 2>/dev/null | grep '^{') || exit 1
    fi
    echo "round $r $v $line" >> $out
  done
done
cat $out
