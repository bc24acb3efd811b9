#!/bin/bash
# This build's attention vs ab_lib/libtdl_kernels_old.so: numerics (all attention GPU tests), then
# interleaved timing at the bench shape, 3 rounds
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/attn_ab2.txt
: > $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_ab2_t.log 2>&1 || { echo "tests failed" >> $out; tail -20 gpurun_out/attn_ab2_t.log; exit 1; }
tail -1 gpurun_out/attn_ab2_t.log >> $out
for r in 1 2 3; do
  line=$(TDL_NATIVE_LIB=$PWD/ab_lib/libtdl_kernels_old.so timeout -k 10 120 python -u scripts/attn_time.py 2>/dev/null | grep '^{') || exit 1
  echo "round $r old $line" >> $out
  line=$(timeout -k 10 120 python -u scripts/attn_time.py 2>/dev/null | grep '^{') || exit 1
  echo "round $r new $line" >> $out
done
cat $out
