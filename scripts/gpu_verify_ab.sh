#!/bin/bash
# Verification overhead, interleaved on one box: bench.py verify on vs --no-verify, GPT-2-small and
# GPT-2-medium, ROUNDS rounds (default 3).  One JSON line per run in gpurun_out/verify_ab.txt.
mkdir -p gpurun_out
out=gpurun_out/verify_ab.txt
: > $out
for r in $(seq 1 ${ROUNDS:-3}); do
  for m in gpt2-small gpt2-medium; do
    for v in on off; do
      extra=""; [ $v = off ] && extra="--no-verify"
      line=$(timeout -k 10 240 python -u bench.py --model $m --steps 10 --warmup 3 $extra 2>/dev/null | grep '^{') || exit 1
      echo "round $r $m verify=$v $line" >> $out
      echo "round $r $m $v done"
    done
  done
done
