#!/bin/bash
# verify on / --no-verify interleaved A/B of the N=1 bench at its defaults (3 + 3 runs)
mkdir -p gpurun_out/vab
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/vab/on_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-verify > gpurun_out/vab/off_$i.json 2>/dev/null || exit 1
  echo "run $i on $(grep -o '"value": [0-9.]*' gpurun_out/vab/on_$i.json) off $(grep -o '"value": [0-9.]*' gpurun_out/vab/off_$i.json)"
done
