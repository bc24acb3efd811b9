#!/bin/bash
# Attention + GPU tests that touch changed kernels (isolated), then bench + rocprof stats.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
SKIP_BENCH=1 PYTEST_TARGET="${PYTEST_TARGET:-tests/test_kernels_gpu.py}" bash scripts/gpu_tests_isolated.sh || exit $?
timeout -k 10 420 python -u bench.py --steps ${BENCH_STEPS:-5} --warmup 2 ${BENCH_ARGS} > gpurun_out/bench1.log 2>&1 || { tail -20 gpurun_out/bench1.log; exit 1; }
grep metric gpurun_out/bench1.log
bash scripts/gpu_profile.sh
