#!/bin/bash
# Round-3 opening measurement: round-end rehearsal (pytest -m gpu, smoke, bench) then a rocprofv3
# kernel-trace profile of a short bench run.  Each GPU step has its own time limit; stop at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/scripts/gpu_roundend.sh || exit $?
mkdir -p $R/gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof/bench.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -2 $R/gpurun_out/prof/bench.log
exit $rc
