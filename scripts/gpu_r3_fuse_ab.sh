#!/bin/bash
# Interleaved bench A/B of the verifier statistics fused into the weight-gradient reduce
# (TDL_FUSED_GRAD_STATS 1) vs the side-stream pass (0), 3 rounds, then the GPU tests that cover it.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "grad_stats or fused or early or attention or flash" > $R/gpurun_out/pytest_fuse_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $R/gpurun_out/pytest_fuse_ab.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for f in 0 1; do
    TDL_FUSED_GRAD_STATS=$f timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > $R/gpurun_out/ab_fuse_${f}_$i.log 2>&1
    rc=$?; echo "fused=$f round $i rc=$rc $(tail -1 $R/gpurun_out/ab_fuse_${f}_$i.log | cut -c1-110)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
