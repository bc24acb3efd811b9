#!/bin/bash
# Run every GPU test in its own process (own timeout, uncaptured output), stop at the first failure,
# then a short N=1 bench.  A fault therefore names its test and nothing runs on the GPU after it.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
LOG=gpurun_out/gpu_tests.log
: > $LOG
TARGET=${PYTEST_TARGET:-tests/test_kernels_gpu.py}
ids=$(python -m pytest $TARGET -m gpu --collect-only -q -p no:cacheprovider 2>/dev/null | grep "::")
for t in $ids; do
  echo "== $t" >> $LOG
  timeout -k 10 ${TEST_TIMEOUT:-180} python -u -m pytest "$t" -x -q -s -p no:cacheprovider >> $LOG 2>&1
  rc=$?
  echo "rc=$rc" >> $LOG
  if [ $rc -eq 1 ]; then FAILED="$FAILED $t"; continue; fi
  if [ $rc -ne 0 ]; then echo "STOP at $t rc=$rc"; tail -40 $LOG; exit $rc; fi
done
grep -c "^rc=0" $LOG; echo "FAILED:$FAILED"
if [ -n "$SKIP_BENCH" ]; then exit 0; fi
timeout -k 10 420 python -u bench.py --steps ${BENCH_STEPS:-5} --warmup 2 ${BENCH_ARGS} > gpurun_out/bench1.log 2>&1
rc2=$?
echo "bench rc=$rc2"; tail -20 gpurun_out/bench1.log
exit $rc2
