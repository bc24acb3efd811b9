#!/bin/bash
# BatchNorm pass microbenchmark (scripts/bench_bn.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out
: > gpurun_out/bn_sweep.jsonl
for b in ${LABELS:-new}; do
  BN_LABEL=$b timeout -k 10 120 python -u scripts/bench_bn.py >> gpurun_out/bn_sweep.jsonl 2> gpurun_out/bn_err.log
  rc=$?; echo "build=$b rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/bn_err.log; exit $rc; }
done
cat gpurun_out/bn_sweep.jsonl
