#!/bin/bash
# One box: CNN path (conv / BN / max-pool GPU tests, ResNet-50 + VGG-16 bench, ResNet-50 kernel profile),
# then the MLP native-vs-library A/B.  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/scripts/gpu_cnn.sh || exit $?
bash $R/scripts/gpu_r3_mlp_ab.sh
