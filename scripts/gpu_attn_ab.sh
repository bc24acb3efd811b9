#!/bin/bash
# Interleaved A/B of two attention builds: old = ab_lib/libtdl_kernels_old.so, new = in-tree (3 rounds)
mkdir -p gpurun_out
out=gpurun_out/attn_ab.txt
: > $out
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export TDL_NATIVE_LIB=$PWD/ab_lib/libtdl_kernels_old.so; else unset TDL_NATIVE_LIB; fi
    line=$(timeout -k 10 120 python -u scripts/attn_time.py 2>/dev/null | grep '^{') || exit 1
    echo "round $r $v $line" >> $out
  done
done
cat $out
