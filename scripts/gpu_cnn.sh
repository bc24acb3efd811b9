#!/bin/bash
# CNN pipeline bench (native conv path) + rocprofv3 kernel stats of a short ResNet-50 run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/prof_cnn
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1 || { tail -30 gpurun_out/pytest_conv.log; exit 1; }
true
timeout -k 10 300 python -u bench_cnn.py --model resnet50 --image-size 224 --batch-per-gpu 64 --steps 5 --warmup 2 > gpurun_out/bench_r50.log 2>&1 || { tail -30 gpurun_out/bench_r50.log; exit 1; }
grep metric gpurun_out/bench_r50.log
timeout -k 10 300 python -u bench_cnn.py --model vgg16 --image-size 224 --batch-per-gpu 32 --steps 5 --warmup 2 > gpurun_out/bench_vgg16.log 2>&1 || { tail -30 gpurun_out/bench_vgg16.log; exit 1; }
grep metric gpurun_out/bench_vgg16.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_cnn -o run -- \
  python3 $R/bench_cnn.py --model resnet50 --image-size 224 --batch-per-gpu 64 --steps 3 --warmup 1 > $R/gpurun_out/prof_cnn/bench.log 2>&1 || exit 1
cd $R && python scripts/prof_summary.py $(find gpurun_out/prof_cnn -name "*kernel_stats.csv" | head -1) 4 30 > gpurun_out/prof_cnn_summary.txt && head -32 gpurun_out/prof_cnn_summary.txt
