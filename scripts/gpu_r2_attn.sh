#!/bin/bash
# Attention after the transposed-read swizzle: numerics (incl. production shape), microbench, LDS PMC.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "attention" > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
timeout -k 10 300 python -u scripts/bench_attn.py > gpurun_out/attn_bench_r2.jsonl 2>&1 || { tail -20 gpurun_out/attn_bench_r2.jsonl; exit 1; }
cat gpurun_out/attn_bench_r2.jsonl | grep '^{'
PROGS="attn_only" PMC_OUT=pmc_attn_r2 timeout -k 10 400 bash scripts/gpu_pmc_attn.sh > gpurun_out/pmc_attn_r2.log 2>&1 || { tail -20 gpurun_out/pmc_attn_r2.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmc_attn_r2 > gpurun_out/pmc_attn_r2_summary.txt 2>&1; head -20 gpurun_out/pmc_attn_r2_summary.txt
