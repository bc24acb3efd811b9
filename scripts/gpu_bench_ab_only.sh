#!/bin/bash
# Interleaved in-step A/B only (no test suite): VARIANTS="a=ENV=1;b=ENV=2" bash scripts/gpu_bench_ab_only.sh
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
bash scripts/gpu_bench_env_ab.sh
