#!/bin/bash
# Forward prefetch depth (TDL_ATTN_FWD_PF 1 | 2: asm two-ahead K/V loads); numerics under both,
# then interleaved timing at the bench shape (3 rounds)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/attn_fwdpf.txt
: > $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_fwdpf_t.log 2>&1 || { echo "tests failed" >> $out; tail -30 gpurun_out/attn_fwdpf_t.log; exit 1; }
TDL_ATTN_FWD_PF=2 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention" -x -q --timeout 120 --timeout-method thread > gpurun_out/attn_fwdpf_t2.log 2>&1 || { echo "tests(pf2) failed" >> $out; tail -30 gpurun_out/attn_fwdpf_t2.log; exit 1; }
for r in 1 2 3; do
  for v in 1 2; do
    line=$(TDL_ATTN_FWD_PF=$v timeout -k 10 120 python -u scripts/attn_time.py 2>/dev/null | grep '^{') || exit 1
    echo "round $r fwd_pf=$v $line" >> $out
  done
done
cat $out
