#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/ab_flags_on.json 2>gpurun_out/ab_flags_on.err || exit 1
timeout -k 10 300 python -u /root/repo/scripts/ab_cpu_gpu.py cuda:0 > gpurun_out/ab_tiny_gpu.txt 2>&1 || exit 1
cat gpurun_out/ab_flags_on.json gpurun_out/ab_tiny_gpu.txt
