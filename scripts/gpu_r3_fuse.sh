#!/bin/bash
# Fused verification reduce + fused qkv-bias gradient: GPU tests, interleaved bench A/B of the fused
# statistics (TDL_FUSED_GRAD_STATS 0/1), kernel-trace profile.  Each GPU step time-limited; stop at first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/prof_fuse
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_conv_gpu.py -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $R/gpurun_out/pytest_fuse.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $R/gpurun_out/pytest_fuse.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for f in 0 1; do
    TDL_FUSED_GRAD_STATS=$f timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > $R/gpurun_out/bench_fuse_${f}_$i.log 2>&1
    rc=$?; echo "bench fused=$f round $i rc=$rc $(tail -1 $R/gpurun_out/bench_fuse_${f}_$i.log | cut -c1-140)"; [ $rc -ne 0 ] && exit $rc
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_fuse -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof_fuse/bench.log 2>&1
rc=$?; echo "prof rc=$rc"
exit $rc
