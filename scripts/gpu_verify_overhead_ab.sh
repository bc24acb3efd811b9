#!/bin/bash
# Verification overhead, interleaved on one box: bench.py defaults with verification on vs --no-verify
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
out=gpurun_out/verify_ab.txt
: > $out
for r in 1 2 3; do
  for v in on off; do
    args=""; [ $v = off ] && args="--no-verify"
    line=$(timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 $args 2>/dev/null | grep '^{') || { echo "round $r $v failed" >> $out; exit 1; }
    val=$(echo "$line" | python -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
    echo "round $r verify=$v value ms/step: $val" >> $out
  done
done
cat $out
