#!/bin/bash
# Kernel-level profile of a short bench run (rocprofv3 kernel trace + stats, no PMC counters).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- \
  python3 $R/bench.py --steps ${BENCH_STEPS:-3} --warmup 1 ${BENCH_ARGS} > $R/gpurun_out/prof/bench.log 2>&1
rc=$?
echo "rc=$rc"; tail -3 $R/gpurun_out/prof/bench.log
find $R/gpurun_out/prof -name "*stats*" | head
exit $rc
