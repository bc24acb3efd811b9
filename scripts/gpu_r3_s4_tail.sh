#!/bin/bash
# BN forward software pipelining: conv GPU tests, BN microbench, ResNet-50 / VGG-16 bench + profile
# (gpu_cnn.sh); then the verification on/off A/B for GPT-2-small and -medium (3 rounds).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd $R && timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k production > gpurun_out/pytest_bnprod.log 2>&1 || { tail -30 gpurun_out/pytest_bnprod.log; exit 1; }
cd $R && LABELS=fwdpipe bash $R/scripts/gpu_r3_bn.sh || exit $?
cd $R && bash $R/scripts/gpu_cnn.sh || exit $?
cd $R && ROUNDS=3 bash $R/scripts/gpu_small_verify_ab.sh
