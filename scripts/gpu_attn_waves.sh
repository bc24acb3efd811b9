#!/bin/bash
# 4- vs 8-wave attention workgroups (TDL_ATTN_WAVES = fwd,dQ,dKdV digits): numerics under the
# all-8 setting and the default, then an interleaved timing A/B at the bench shape (3 rounds)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/attn_waves.txt
: > $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_waves_t4.log 2>&1 || { echo "tests(default) failed" >> $out; exit 1; }
TDL_ATTN_WAVES=8 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_waves_t8.log 2>&1 || { echo "tests(8) failed" >> $out; exit 1; }
for r in 1 2 3; do
  for v in ${VARIANTS:-444 844 884 848}; do
    line=$(TDL_ATTN_WAVES=$v timeout -k 10 120 python -u scripts/attn_time.py 2>/dev/null | grep '^{') || exit 1
    echo "round $r waves=$v $line" >> $out
  done
done
cat $out
