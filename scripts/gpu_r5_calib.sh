#!/bin/bash
# Round 5: clean GPT-2-medium reference curve (full flow, no attack) + configs 3 / dx re-run after
# the GC-free re-shard (migration estimate check), 3 seeds each.
mkdir -p gpurun_out
CFGS=clean,3,dx SEEDS=1,2,3 STEPS=170 MODE=full OUT=gpurun_out/r5_cfg_calib.jsonl CFG_TIMEOUT=1120 bash scripts/gpu_r4_configs.sh
