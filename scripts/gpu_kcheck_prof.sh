#!/bin/bash
# Kernel numerics (all GPU kernel tests), N=1 bench, then a rocprofv3 kernel-stats pass (TAG).
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${TAG:-v12}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_block.py tests/test_fwd_weight_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/kcheck_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/kcheck_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/kcheck_bench.log 2>&1 || { tail -20 gpurun_out/kcheck_bench.log; exit 1; }
grep metric gpurun_out/kcheck_bench.log | cut -c1-200
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 1; }
f=$(find $R/gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
python3 $R/scripts/prof_summary.py "$f" 7 40 > $R/gpurun_out/prof_${TAG}_summary.txt
grep -E "total|attn_delta|transpose|xent" $R/gpurun_out/prof_${TAG}_summary.txt
