#!/bin/bash
# GPT-2 kernel tests + N=1 bench at the default and at pipeline-size micro-batches.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_block.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_k.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_k.log; [ $rc -ne 0 ] && exit $rc
for m in ${MBS_LIST:-32 8}; do
  timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --mbs $m ${BENCH_ARGS} > gpurun_out/bench_mbs$m.log 2>&1 || { tail -20 gpurun_out/bench_mbs$m.log; exit 1; }
  echo "mbs=$m $(grep metric gpurun_out/bench_mbs$m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
