#!/bin/bash
# N=1 bench: micro-batch 32 (2 micro-batches, the default) vs 64 (one micro-batch), interleaved.
mkdir -p gpurun_out/mbs
for i in 1 2; do
  for m in 32 64; do
    timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --mbs $m > gpurun_out/mbs/b_${m}_${i}.log 2>&1 || exit $?
    echo "mbs=$m run=$i $(grep -o '"value": [0-9.]*' gpurun_out/mbs/b_${m}_${i}.log)"
  done
done
