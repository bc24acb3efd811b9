#!/bin/bash
# Integrity checksum overlapped on the side stream + no unused quantile histograms: whole GPU suite,
# then the verification on/off A/B for GPT-2-small / -medium (3 rounds).  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_all_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_all_gpu.log; [ $rc -ne 0 ] && exit $rc
ROUNDS=3 bash $R/scripts/gpu_small_verify_ab.sh
