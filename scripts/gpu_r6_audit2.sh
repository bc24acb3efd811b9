#!/bin/bash
# Round 6: audit kernels + GPU protocol tests, the protocol's cost (interleaved off / fwd / mirror),
# and the weight-gradient split-K sweep at the engine's token counts.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_audit_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/audit_kernels_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/audit_kernels_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/wgrad_split_sweep.py --out gpurun_out/r6_wgrad_split_sweep.jsonl > gpurun_out/wgrad_sweep.log 2>&1
rc=$?; grep best_split gpurun_out/wgrad_sweep.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u scripts/audit_overhead.py --steps 6 --warmup 2 --rounds 2 --out gpurun_out/r6_audit_overhead_v2.jsonl
