#!/bin/bash
# Round 6: the whole GPU test tier, then a kernel-level profile of the full audit protocol
# (GPT-2-medium, 8 stages local mode on one GPU, M = 16).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/prof_audit
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "${SKIP_TESTS:-0}" != "1" ]; then
timeout -k 10 900 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > $R/gpurun_out/pytest_all_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 $R/gpurun_out/pytest_all_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_audit -o run -- \
  python3 $R/scripts/audit_overhead.py --variants ${VARIANTS:-mirror} --steps 3 --warmup 1 --rounds 1 --out $R/gpurun_out/prof_audit/ov.jsonl > $R/gpurun_out/prof_audit/log.txt 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 $R/gpurun_out/prof_audit/log.txt
exit $rc
