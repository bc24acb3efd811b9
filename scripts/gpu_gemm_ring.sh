#!/bin/bash
# Ring ping-pong GEMM (gemm_pr): GPU tests, then tile-order x kernel A/B vs hipBLASLt and the in-kernel timeline.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/ring
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q -k "ring or epilogues or layouts or fused_mlp" --timeout 120 --timeout-method thread > $R/gpurun_out/ring/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $R/gpurun_out/ring/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/gemm_order_ab.py --kernels pp,pr --groups 0,8 ${AB_ARGS} > $R/gpurun_out/ring/order_ab.jsonl 2> $R/gpurun_out/ring/order_ab.err
rc=$?; echo "order_ab rc=$rc"; cat $R/gpurun_out/ring/order_ab.jsonl; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/ring/order_ab.err; exit $rc; }
timeout -k 10 200 python -u scripts/gemm_order_ab.py --kernels pp,pr --groups 8 --epi gelu --only fc_fwd > $R/gpurun_out/ring/order_ab_gelu.jsonl 2>> $R/gpurun_out/ring/order_ab.err
rc=$?; echo "gelu rc=$rc"; cat $R/gpurun_out/ring/order_ab_gelu.jsonl; [ $rc -ne 0 ] && exit $rc
TDL_GEMM_GROUPM=8 timeout -k 10 200 python -u scripts/gemm_timeline.py --kernels pp,pr > $R/gpurun_out/ring/timeline.jsonl 2> $R/gpurun_out/ring/timeline.err
rc=$?; echo "timeline rc=$rc"; cat $R/gpurun_out/ring/timeline.jsonl
exit $rc
