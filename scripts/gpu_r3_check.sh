#!/bin/bash
# GEMM GPU tests + short bench + kernel-trace profile (each step time-limited; stop at first failure)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $R/gpurun_out/pytest_gemm.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $R/gpurun_out/pytest_gemm.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > $R/gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $R/gpurun_out/bench.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof/bench.log 2>&1
rc=$?; echo "prof rc=$rc"
exit $rc
