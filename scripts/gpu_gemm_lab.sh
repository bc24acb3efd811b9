#!/bin/bash
# GEMM lab on the GPU: fp32 checks of both native kernels, then the GPT-2-medium products vs hipBLASLt.
mkdir -p gpurun_out
timeout -k 10 ${LAB_TIMEOUT:-500} python -u scripts/gemm_lab.py ${LAB_ARGS} > gpurun_out/gemm_lab.log 2>&1
rc=$?; echo "lab rc=$rc"; grep -v '"check"' gpurun_out/gemm_lab.log | grep -c worst; grep '"check"\|product\|Error\|error' gpurun_out/gemm_lab.log | tail -30
exit $rc
