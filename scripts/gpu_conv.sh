#!/bin/bash
# Conv/BN kernel numerics, then the conv microbenchmark (native vs MIOpen).
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_conv.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/bench_conv.py > gpurun_out/bench_conv.log 2>&1
rc=$?
echo "bench_conv rc=$rc"; cat gpurun_out/bench_conv.log | tail -20
exit $rc
