#!/bin/bash
# Interleaved bench A/B: the step on a high-priority HIP stream (TDL_COMPUTE_PRIORITY=high) vs the
# default stream, with the verification side stream at default priority in both.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2 3; do
  for f in default high; do
    TDL_COMPUTE_PRIORITY=$f timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > $R/gpurun_out/ab_prio_${f}_$i.log 2>&1
    rc=$?; echo "priority=$f round $i rc=$rc $(tail -1 $R/gpurun_out/ab_prio_${f}_$i.log | cut -c1-110)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
