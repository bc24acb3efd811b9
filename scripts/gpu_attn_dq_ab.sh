#!/bin/bash
# dQ staging depth: TDL_ATTN_DQ_PF=2 (one 32-key half at a time + two K/V register sets) vs 1;
# numerics under PF=2, then interleaved timing (3 rounds)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/attn_dq_ab.txt
: > $out
TDL_ATTN_DQ_PF=2 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_dq_t.log 2>&1 || { echo "tests failed" >> $out; tail -20 gpurun_out/attn_dq_t.log; exit 1; }
tail -1 gpurun_out/attn_dq_t.log >> $out
for r in 1 2 3; do
  for v in 1 2; do
    line=$(TDL_ATTN_DQ_PF=$v timeout -k 10 120 python -u scripts/attn_time.py 2>/dev/null | grep '^{') || exit 1
    echo "round $r dq_pf=$v $line" >> $out
  done
done
cat $out
