#!/bin/bash
# Host-side view of the GPT-2-medium step: HIP API trace + kernel trace of a short bench run (where
# does the host block, how far ahead of the GPU is it at the step tail).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/ht && cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d $R/gpurun_out/ht -o run -- \
  python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/ht/bench.log 2>&1
rc=$?; echo "hiptrace rc=$rc"; ls -la $R/gpurun_out/ht
exit $rc
