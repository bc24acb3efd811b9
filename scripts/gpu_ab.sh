#!/bin/bash
# A/B of an env toggle on the N=1 headline bench, interleaved on one box: A B A B.
# usage: AB_ENV="TDL_FUSED_LMHEAD=0" bash scripts/gpu_ab.sh
mkdir -p gpurun_out
for k in 1 2; do
  for arm in A B; do
    if [ $arm = B ]; then envs="$AB_ENV"; else envs=""; fi
    env $envs timeout -k 10 300 python -u bench.py --steps ${STEPS:-8} --warmup 3 ${BENCH_ARGS} > gpurun_out/ab_$arm$k.log 2>&1 || { tail -5 gpurun_out/ab_$arm$k.log; exit 1; }
    echo "$arm$k $(grep -o '"value": [0-9.]*' gpurun_out/ab_$arm$k.log)"
  done
done
