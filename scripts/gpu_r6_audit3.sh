#!/bin/bash
# Round 6: protocol cost, each (round, variant) in its own process, interleaved; then the LM-head
# weight-gradient split sweep (validates the split cost model on the tied head).
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u scripts/audit_overhead.py --steps 6 --warmup 2 --rounds 2 --out gpurun_out/r6_audit_overhead_v3.jsonl || exit 1
timeout -k 10 200 python -u scripts/wgrad_split_sweep.py --products lmhead --Ks 16384,65536 --out gpurun_out/r6_wgrad_split_sweep_lmhead.jsonl > gpurun_out/wgrad_sweep_lm.log 2>&1
rc=$?; grep best_split gpurun_out/wgrad_sweep_lm.log; exit $rc
