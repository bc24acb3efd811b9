#!/bin/bash
# Store-first staging A/B: old build (ab_lib/libtdl_kernels_old.so) vs this build (dK/dV PF 2 and
# the store-first PF 1); numerics of this build first; interleaved timing, 3 rounds
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/attn_sf_ab.txt
: > $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_sf_t.log 2>&1 || { echo "tests failed" >> $out; tail -20 gpurun_out/attn_sf_t.log; exit 1; }
TDL_ATTN_DKDV_PF=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_sf_t1.log 2>&1 || { echo "tests(pf1) failed" >> $out; tail -20 gpurun_out/attn_sf_t1.log; exit 1; }
for r in 1 2 3; do
  line=$(TDL_NATIVE_LIB=$PWD/ab_lib/libtdl_kernels_old.so timeout -k 10 120 python -u scripts/attn_time.py 2>/dev/null | grep '^{') || exit 1
  echo "round $r old $line" >> $out
  line=$(timeout -k 10 120 python -u scripts/attn_time.py 2>/dev/null | grep '^{') || exit 1
  echo "round $r new(pf2) $line" >> $out
  line=$(TDL_ATTN_DKDV_PF=1 timeout -k 10 120 python -u scripts/attn_time.py 2>/dev/null | grep '^{') || exit 1
  echo "round $r new(pf1-sf) $line" >> $out
done
cat $out
