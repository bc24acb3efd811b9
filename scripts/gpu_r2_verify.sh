#!/bin/bash
# Round-2 verification-overlap checks: GPU tests for the split K3 pass, then an interleaved
# verify-on / verify-off bench A/B (N=1, GPT-2-medium headline config).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_conv_gpu.py > gpurun_out/r2_tests.log 2>&1
rc=$?; tail -5 gpurun_out/r2_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/ab_on_$i.json 2> gpurun_out/ab_on_$i.err || exit 1
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-verify > gpurun_out/ab_off_$i.json 2> gpurun_out/ab_off_$i.err || exit 1
done
cat gpurun_out/ab_*.json
