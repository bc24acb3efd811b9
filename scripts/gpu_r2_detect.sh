#!/bin/bash
# Round-2 detection-under-learning measurements on one MI355X (local multi-stage mode).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u bench_detection.py --part protocol --out gpurun_out/det_protocol.json > gpurun_out/det_protocol.log 2>&1 || { tail -20 gpurun_out/det_protocol.log; exit 1; }
timeout -k 10 600 python -u bench_detection.py --part fp --data markov --data-vocab 8192 --lr-warmup 50 --steps 500 --warm 50 --lr 1e-4 --out gpurun_out/det_fp_markov.json > gpurun_out/det_fp.log 2>&1 || { tail -20 gpurun_out/det_fp.log; exit 1; }
grep '"fp"' gpurun_out/det_fp.log | cut -c1-400
timeout -k 10 900 python -u bench_detection.py --part engine --data markov --data-vocab 8192 --lr-warmup 50 --steps 200 --warm 100 --lr 1e-4 --out gpurun_out/det_engine_markov.json > gpurun_out/det_engine.log 2>&1 || { tail -20 gpurun_out/det_engine.log; exit 1; }
grep '^{' gpurun_out/det_engine.log | cut -c1-300
timeout -k 10 900 python -u scripts/run_attack_configs.py --configs 3,4,5 --out gpurun_out/attack_configs.jsonl > gpurun_out/attack_configs.log 2>&1 || { tail -20 gpurun_out/attack_configs.log; exit 1; }
grep -c '^{' gpurun_out/attack_configs.log
