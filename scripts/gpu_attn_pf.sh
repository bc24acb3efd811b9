#!/bin/bash
# Prefetch depth of the attention backward kernels: TDL_ATTN_DKDV_PF (2 | 3) and TDL_ATTN_DQ_PF
# (1 | 2); numerics under the deepest setting, then interleaved timing at the bench shape (3 rounds)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/attn_pf.txt
: > $out
TDL_ATTN_DKDV_PF=3 TDL_ATTN_DQ_PF=2 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_pf_t.log 2>&1 || { echo "tests failed" >> $out; tail -20 gpurun_out/attn_pf_t.log; exit 1; }
for r in 1 2 3; do
  for v in "2 1" "3 1" "2 2" "3 2"; do
    set -- $v
    line=$(TDL_ATTN_DKDV_PF=$1 TDL_ATTN_DQ_PF=$2 timeout -k 10 120 python -u scripts/attn_time.py 2>/dev/null | grep '^{') || exit 1
    echo "round $r dkdv_pf=$1 dq_pf=$2 $line" >> $out
  done
done
cat $out
