#!/bin/bash
# rocprofv3 kernel stats of the N=1 bench at its current defaults (micro-batch 64, one micro-batch):
# 3 timed + 2 warm-up steps = 5 steps in the table.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/prof_r2b
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r2b -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_r2b/bench.log 2>&1 || { tail -20 $R/gpurun_out/prof_r2b/bench.log; exit 1; }
cd $R
TR=$(find gpurun_out/prof_r2b -name "*kernel_trace.csv" | head -1)
ST=$(find gpurun_out/prof_r2b -name "*kernel_stats.csv" | head -1)
python scripts/overlap_from_trace.py $TR > gpurun_out/prof_r2b/overlap.json && cat gpurun_out/prof_r2b/overlap.json
python scripts/prof_summary.py $ST 5 40 > gpurun_out/prof_r2b/summary.txt && head -45 gpurun_out/prof_r2b/summary.txt
rm -f $TR
