#!/bin/bash
# Round 6: protocol cost after the tail-sync fix and batched commitment trees: host profiles of off and
# mirror, then interleaved isolated runs (off / fwd / mirror x 2 rounds), then the GPU audit tests.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in off mirror; do
  timeout -k 10 300 python -u scripts/audit_overhead.py --inproc --variants $v --steps 3 --warmup 2 --cprofile gpurun_out/cprof5 --out gpurun_out/ov_cprof5.jsonl || exit 1
done
timeout -k 10 1000 python -u scripts/audit_overhead.py --steps 6 --warmup 2 --rounds 2 --out gpurun_out/r6_audit_overhead_v5.jsonl || exit 1
timeout -k 10 400 python -u -m pytest tests/test_audit_kernels_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/audit_kernels_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/audit_kernels_gpu.log; exit $rc
