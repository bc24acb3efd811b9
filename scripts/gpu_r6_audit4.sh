#!/bin/bash
# Round 6: host syncs of the local-mode protocol step, then kernel-time sums of off vs mirror.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/prof_off $R/gpurun_out/prof_mir
export HSA_ENABLE_IPC_MODE_LEGACY=0
PROBE_MODULE=scripts.audit_overhead timeout -k 10 400 python -u scripts/sync_probe.py --inproc --variants mirror --steps 2 --warmup 1 --out $R/gpurun_out/sync_probe.jsonl > $R/gpurun_out/sync_probe.log 2>&1 || { tail -20 $R/gpurun_out/sync_probe.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
for v in off mirror; do
  d=$R/gpurun_out/prof_${v:0:3}
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
    python3 $R/scripts/audit_overhead.py --inproc --variants $v --steps 3 --warmup 1 --out $d/ov.jsonl > $d/log.txt 2>&1 || { tail -5 $d/log.txt; exit 1; }
done
echo ok
