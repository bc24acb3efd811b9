#!/bin/bash
# Round 6: protocol cost after the LDS-staged leaf hash and the cross-member tie check: interleaved
# isolated runs (off / fwd / mirror x 2 rounds), GPT-2-medium, 8 stages in local mode, M = 16.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u scripts/audit_overhead.py --steps 6 --warmup 2 --rounds 2 --out gpurun_out/r6_audit_overhead_v6.jsonl
