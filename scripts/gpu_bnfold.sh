#!/bin/bash
# ResNet-50 224 batch 64 (bench_cnn.py, N=1): BN fold on / off interleaved (3 + 3 runs), then a
# rocprofv3 kernel-stats pass of the folded path.  Each GPU step has its own time limit.
mkdir -p gpurun_out/bnfold
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2; do
  for f in 1 0; do
    TDL_BN_FOLD=$f timeout -k 10 200 python -u bench_cnn.py --model resnet50 --steps 10 --warmup 3 > gpurun_out/bnfold/run_${f}_${i}.log 2>&1 || exit $?
    echo "fold=$f run=$i $(grep -o '"value": [0-9.]*' gpurun_out/bnfold/run_${f}_${i}.log)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TDL_BN_FOLD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bnfold/prof --output-format csv -o run -- python3 bench_cnn.py --model resnet50 --steps 4 --warmup 2 > gpurun_out/bnfold/prof.log 2>&1 || exit $?
find gpurun_out/bnfold/prof -name "*kernel_stats.csv" | head -3
