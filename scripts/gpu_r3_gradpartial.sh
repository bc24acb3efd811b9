#!/bin/bash
# Verification partial pass with one shift per chunk (plain block sums): GPU stats tests, bench x3,
# kernel-trace profile of the bench (side stream) and of a serialized run (TDL_SERIALIZE_STREAMS=1:
# the pass on the compute stream, i.e. its isolated kernel time).  Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/gp
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "grad_stats or early_grad or verify or fused" > gpurun_out/gp/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gp/pytest.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/gp/bench_$i.log 2>&1
  rc=$?; echo "bench $i rc=$rc $(tail -1 gpurun_out/gp/bench_$i.log | cut -c1-120)"; [ $rc -ne 0 ] && exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/gp/prof -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/gp/prof_bench.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
export TDL_SERIALIZE_STREAMS=1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/gp/prof_ser -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/gp/prof_ser_bench.log 2>&1
rc=$?; echo "prof serialized rc=$rc"
exit $rc
