#!/bin/bash
# GPU validation run: kernel numerics (uncaptured, verbose, so a fault message is never swallowed),
# then a short bench.  Each GPU step has its own timeout; stop at the first failure.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest ${PYTEST_TARGET:-tests/test_kernels_gpu.py} -x -v -s -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps ${BENCH_STEPS:-5} --warmup 2 ${BENCH_ARGS} > gpurun_out/bench1.log 2>&1
rc2=$?
echo "bench rc=$rc2"; tail -20 gpurun_out/bench1.log
exit $rc2
