#!/bin/bash
# Round 5: audit kernels vs host, then the adaptive-adversary configs (detection only: every
# injection scored) on GPT-2-medium, 8 stages on one MI355X, M = 16 micro-batches.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u -m pytest tests/test_audit_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/audit_kernels_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/audit_kernels_gpu.log; [ $rc -ne 0 ] && exit $rc
CFGS=3a SEEDS=1,2,3 STEPS=170 MODE=detect OUT=gpurun_out/r5_cfg_adaptive.jsonl CFG_TIMEOUT=500 bash scripts/gpu_r4_configs.sh || exit 1
CFGS=3am SEEDS=1,2,3 STEPS=300 MODE=detect OUT=gpurun_out/r5_cfg_adaptive.jsonl CFG_TIMEOUT=600 bash scripts/gpu_r4_configs.sh
