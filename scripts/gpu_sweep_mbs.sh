#!/bin/bash
# N=1 bench at several micro-batch sizes (same global batch): GEMM/attention efficiency vs bubble.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for m in ${MBS_LIST:-4 8 16 32}; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --mbs $m ${BENCH_ARGS} > gpurun_out/sweep_mbs$m.log 2>&1 || { tail -20 gpurun_out/sweep_mbs$m.log; exit 1; }
  echo "mbs=$m $(grep metric gpurun_out/sweep_mbs$m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
