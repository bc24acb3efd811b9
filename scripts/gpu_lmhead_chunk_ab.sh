#!/bin/bash
# LM-head logits budget A/B on the N=1 bench (interleaved): 4096 MB (whole micro-batch of 32 x 1024
# rows, 3.3 GB of logits) vs 1024 / 512 MB chunks (logits never materialised beyond the budget).
mkdir -p gpurun_out/lmchunk
for i in 1 2; do
  for mb in 4096 1024 512; do
    TDL_LMHEAD_CHUNK_MB=$mb timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/lmchunk/b_${mb}_${i}.log 2>&1 || exit $?
    echo "budget=${mb}MB run=$i $(grep -o '"value": [0-9.]*' gpurun_out/lmchunk/b_${mb}_${i}.log)"
  done
done
