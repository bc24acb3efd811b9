#!/bin/bash
# BN microbench sweep, then the CNN path (conv GPU tests, ResNet-50 / VGG-16 bench, ResNet-50 profile).
R=${GRAFT_REPO_ROOT:-$(pwd)}
bash $R/scripts/gpu_r3_bn.sh || exit $?
cd $R && bash $R/scripts/gpu_cnn.sh
