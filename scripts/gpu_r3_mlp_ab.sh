#!/bin/bash
# Interleaved bench A/B with the tuned library GEMMs: the MLP's fused-epilogue products on the native
# ping-pong kernel (TDL_MLP_NATIVE=1, default) vs library GEMM + separate bias-GELU passes (0).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2 3; do
  for f in 1 0; do
    TDL_MLP_NATIVE=$f timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > $R/gpurun_out/ab_mlp_${f}_$i.log 2>&1
    rc=$?; echo "mlp_native=$f round $i rc=$rc $(tail -1 $R/gpurun_out/ab_mlp_${f}_$i.log | cut -c1-110)"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
