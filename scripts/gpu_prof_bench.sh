#!/bin/bash
# rocprofv3 kernel-trace stats of the N=1 headline bench (5 steps) + per-kernel summary.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-v7}
MBS=${MBS:-32}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 5 --warmup 2 --mbs $MBS > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
f=$(find $R/gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
python3 $R/scripts/prof_summary.py "$f" 7 > $R/gpurun_out/prof_${TAG}_summary.txt
head -40 $R/gpurun_out/prof_${TAG}_summary.txt
grep metric $R/gpurun_out/prof_$TAG.log
