#!/bin/bash
# Round 6: the BLAKE2s / keyed-sketch / contribution kernels against the host references, the GPU
# local-mode protocol (clean + lying stages), then the protocol's cost on GPT-2-medium (8 stages in
# local mode on one MI355X, M = 16): off / forward-only / full mirror protocol, interleaved.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_audit_kernels_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/audit_kernels_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/audit_kernels_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u scripts/audit_overhead.py --steps ${OV_STEPS:-6} --warmup 2 --rounds ${OV_ROUNDS:-1} --out gpurun_out/r6_audit_overhead.jsonl
