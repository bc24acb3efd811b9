#!/bin/bash
# grouped qkv + o weight-gradient launch: numerics, microbench, in-step A/B (one box)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gemm_gpu.py -k "grouped or production_wgrad or pd_transposed" > gpurun_out/grouped_tests.log 2>&1 \
  && tail -3 gpurun_out/grouped_tests.log \
  && timeout -k 10 300 python -u scripts/wgrad_grouped_ab.py --out gpurun_out/r6_wgrad_grouped_ab.jsonl \
  && timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
     tests/test_engine_gpu.py tests/test_fwd_weight_gpu.py > gpurun_out/grouped_engine_tests.log 2>&1 \
  && tail -3 gpurun_out/grouped_engine_tests.log \
  && VARIANTS="${VARIANTS:-sep=TDL_WGRAD_GROUPED=0;grp=TDL_WGRAD_GROUPED=1}" bash scripts/gpu_bench_env_ab.sh
