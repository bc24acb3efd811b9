#!/bin/bash
# HW-queue false-dependency probe at several GPU_MAX_HW_QUEUES settings (one process each).
mkdir -p gpurun_out
for q in default 8 16 32; do
  if [ "$q" = default ]; then
    timeout -k 10 90 python -u scripts/hwqueue_probe.py --out gpurun_out/hwq_$q.json || exit $?
  else
    GPU_MAX_HW_QUEUES=$q timeout -k 10 90 python -u scripts/hwqueue_probe.py --out gpurun_out/hwq_$q.json || exit $?
  fi
done
