#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out && rm -f gpurun_out/attack_configs.jsonl
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1000 python -u scripts/run_attack_configs.py --configs 3,4,5 --out gpurun_out/attack_configs.jsonl > gpurun_out/attack_configs.log 2>&1 || { tail -20 gpurun_out/attack_configs.log; exit 1; }
grep -c '^{' gpurun_out/attack_configs.log
