#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PROBE_MODULE=bench_cnn timeout -k 10 300 python -u scripts/op_probe.py --model resnet50 --image-size 224 --batch-per-gpu 64 --steps 3 --warmup 2 > gpurun_out/opprobe_cnn.log 2>&1
rc=$?; echo "probe rc=$rc"; exit $rc
