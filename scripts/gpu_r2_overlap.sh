#!/bin/bash
# rocprof kernel trace of the N=1 bench (verification overlap evidence + per-kernel table), then an
# interleaved verify-on / verify-off A/B of bench.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/prof_r2
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r2 -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_r2/bench.log 2>&1 || { tail -20 $R/gpurun_out/prof_r2/bench.log; exit 1; }
cd $R
TR=$(find gpurun_out/prof_r2 -name "*kernel_trace.csv" | head -1)
ST=$(find gpurun_out/prof_r2 -name "*kernel_stats.csv" | head -1)
python scripts/overlap_from_trace.py $TR > gpurun_out/overlap_r2.json && cat gpurun_out/overlap_r2.json
python scripts/prof_summary.py $ST 5 40 > gpurun_out/prof_r2_summary.txt && head -45 gpurun_out/prof_r2_summary.txt
rm -f $TR
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/ab2_on_$i.json 2>/dev/null || exit 1
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-verify > gpurun_out/ab2_off_$i.json 2>/dev/null || exit 1
done
for f in gpurun_out/ab2_*.json; do echo $f $(python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['config']['detections'], d['config']['last_loss'])"); done
