#!/bin/bash
# GEMM diagnosis: tile-order A/B vs hipBLASLt, then PMC passes (L2 hit rate, wait / busy cycles)
# for the native kernel at two tile orders and the library on the qkv forward product.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/gdiag
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u $R/scripts/gemm_order_ab.py ${AB_ARGS} > $R/gpurun_out/gdiag/order_ab.jsonl 2> $R/gpurun_out/gdiag/order_ab.err
rc=$?; echo "order_ab rc=$rc"; cat $R/gpurun_out/gdiag/order_ab.jsonl; [ $rc -ne 0 ] && { tail -20 $R/gpurun_out/gdiag/order_ab.err; exit $rc; }
cd /tmp && export TMPDIR=/tmp
i=0
for set in "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  for g in 0 8; do
    TDL_GEMM_GROUPM=$g timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/gdiag/pmc_g${g}_p$i -o run -- python3 $R/scripts/gemm_pmc_driver.py > $R/gpurun_out/gdiag/pmc_g${g}_p$i.log 2>&1 || { echo "pmc pass $i g$g failed"; tail -5 $R/gpurun_out/gdiag/pmc_g${g}_p$i.log; exit 1; }
  done
done
echo pmc done
