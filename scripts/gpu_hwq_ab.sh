#!/bin/bash
# N=1 bench with the engine's hardware-queue request vs the box default, interleaved.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 > gpurun_out/hwq_ab_req_$r.log 2>&1 || { tail -20 gpurun_out/hwq_ab_req_$r.log; exit 1; }
  TDL_KEEP_HW_QUEUES=1 timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 > gpurun_out/hwq_ab_keep_$r.log 2>&1 || { tail -20 gpurun_out/hwq_ab_keep_$r.log; exit 1; }
done
grep -h metric gpurun_out/hwq_ab_*.log | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d["config"]["hw_queues"], d["value"], d["ms_per_step"])'
