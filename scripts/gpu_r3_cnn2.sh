#!/bin/bash
# CNN path after the stats-zeroing / materialize changes: conv GPU tests + benches + profile
# (gpu_cnn.sh), then the op-site probe.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && bash $R/scripts/gpu_cnn.sh || exit $?
cd $R && bash $R/scripts/gpu_r3_opprobe.sh
