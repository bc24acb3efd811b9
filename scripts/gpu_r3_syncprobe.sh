#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/sync_probe.py --steps 3 --warmup 2 > gpurun_out/syncprobe.log 2>&1
rc=$?; echo "probe rc=$rc"; exit $rc
