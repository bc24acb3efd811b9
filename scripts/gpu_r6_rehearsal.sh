#!/bin/bash
# Round-6 rehearsal: the driver's round-end tiers (pytest -m gpu, smoke, bench defaults), then a
# rocprofv3 kernel-trace profile of a short bench run.  Each GPU step has its own time limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash scripts/gpu_roundend.sh || exit $?
BENCH_STEPS=3 bash scripts/gpu_profile.sh
