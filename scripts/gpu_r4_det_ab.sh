#!/bin/bash
# Interleaved A/B of the deterministic BN reductions (conv statistics finalize + BN backward fold:
# fixed-order last-workgroup sums instead of fp32 atomics): ResNet-50 bench_cnn, 3 rounds.
#   old = ab_lib/libtdl_kernels_old.so (HEAD before the change), new = the in-tree build
mkdir -p gpurun_out
out=gpurun_out/r4_det_ab.txt
: > $out
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export TDL_NATIVE_LIB=$PWD/ab_lib/libtdl_kernels_old.so; else unset TDL_NATIVE_LIB; fi
    line=$(timeout -k 10 200 python -u bench_cnn.py --model resnet50 --steps 30 --warmup 5 2>/dev/null | grep '^{') || exit 1
    echo "round $r $v $line" >> $out
    echo "round $r $v done"
  done
done
