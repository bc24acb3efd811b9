#!/bin/bash
# Interleaved A/B of environment settings on the ResNet-50 bench (bench_cnn.py), ROUNDS rounds;
# BENCH="bench.py" runs the GPT-2-medium headline bench instead.
#   ENVS="A=1 A=2" OUT=gpurun_out/x.txt bash scripts/gpu_cnn_env_ab.sh
mkdir -p gpurun_out
out=${OUT:-gpurun_out/cnn_env_ab.txt}
: > $out
for r in $(seq 1 ${ROUNDS:-3}); do
  for e in $ENVS; do
    # AB_DIR=<dir>: run that tree (e.g. a build of the previous commit in ab_old/) instead
    dir=.
    case $e in AB_DIR=*) dir=${e#AB_DIR=} ;; esac
    line=$(cd $dir && env $e timeout -k 10 200 python -u ${BENCH:-bench_cnn.py --model ${MODEL:-resnet50}} --steps ${STEPS:-30} --warmup 5 2>/dev/null | grep '^{') || exit 1
    echo "round $r $e $line" >> $out
    echo "round $r $e done"
  done
done
