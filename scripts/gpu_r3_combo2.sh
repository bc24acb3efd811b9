#!/bin/bash
# One box: round-end rehearsal (whole pytest -m gpu suite, smoke, bench defaults), a kernel-trace
# profile of the GPT-2 bench, then the CNN path (ResNet-50 / VGG-16 bench + ResNet-50 profile).
# Each GPU step time-limited (inside the called scripts); stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/scripts/gpu_r3_baseline.sh || exit $?
cd $R && bash $R/scripts/gpu_cnn.sh
