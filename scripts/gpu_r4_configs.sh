#!/bin/bash
# Round-4 attack configurations on one MI355X (local mode, 8 stages on one GPU).
#   CFGS="3s,dx" SEEDS="1,2,3" MODE=detect|full OUT=gpurun_out/r4_cfg.jsonl bash scripts/gpu_r4_configs.sh
# GPT-2-medium at batch 32 / micro-batch 2 (M = 16 micro-batches); ResNet-50 keeps its 64 / 8.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
extra=""
[ "${MODE:-detect}" = "detect" ] && extra="--no-reassign"
timeout -k 10 ${CFG_TIMEOUT:-1100} python -u scripts/run_attack_configs.py --configs "${CFGS}" --seeds "${SEEDS:-1,2,3}" \
    --steps ${STEPS:-300} --start 100 --batch ${BATCH:-32} --mbs ${MBS:-2} --p-attack ${PATTACK:-0.3} $extra \
    --out "${OUT:-gpurun_out/r4_cfg.jsonl}" > gpurun_out/r4_cfg_stdout.log
