#!/bin/bash
# Rehearsal of the driver's round-end GPU tiers: the whole `pytest -m gpu` suite in one process,
# smoke(), then bench.py with its defaults.  Each GPU step has its own time limit; stop at the first failure.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_all_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_all_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench_default.log
exit $rc
