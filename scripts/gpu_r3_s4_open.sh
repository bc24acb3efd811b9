#!/bin/bash
# Session-4 opening: round-end rehearsal + kernel-trace profile (gpu_r3_baseline.sh), then the
# compute-stream priority A/B (gpu_r3_prio_ab.sh).  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/scripts/gpu_r3_baseline.sh || exit $?
cd $R && bash $R/scripts/gpu_r3_prio_ab.sh
