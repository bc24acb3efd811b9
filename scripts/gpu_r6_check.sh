#!/bin/bash
# Round-6 change check: the whole GPU suite (one process), then an interleaved in-step A/B of the
# LM-head dX routing (gemm_pd over the transposed weight copy vs the library GEMM).
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r6.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu_r6.log; [ $rc -ne 0 ] && exit $rc
VARIANTS="${VARIANTS:-pd=TDL_LMHEAD_DX=pd;lib=TDL_LMHEAD_DX=lib}" bash scripts/gpu_bench_env_ab.sh
