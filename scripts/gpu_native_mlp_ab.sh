#!/bin/bash
# Interleaved full-step A/B of the GPT-2-medium N=1 bench: library GEMMs (TDL_NATIVE_GEMM=off) vs
# the native MLP products with fused GELU / dGELU epilogues (mlp) vs every block product native (all).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
out=gpurun_out/native_mlp_ab.txt
: > $out
for round in 1 2 3; do
  for mode in off mlp all; do
    TDL_NATIVE_GEMM=$mode timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/ab_$mode.json 2> gpurun_out/ab_$mode.err || { echo "mode $mode failed"; tail -5 gpurun_out/ab_$mode.err; exit 1; }
    echo "round $round mode $mode $(tail -1 gpurun_out/ab_$mode.json)" >> $out
    tail -1 $out
  done
done
