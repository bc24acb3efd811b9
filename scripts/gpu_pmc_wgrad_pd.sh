#!/bin/bash
# PMC passes (one counter group per run) over the qkv weight gradient on gemm_p4 (TT), gemm_pd (TT)
# and gemm_pd on pre-transposed operands (NT): why the LDS-DMA kernel is fast on NT and slow on TT.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/pmc_wgrad_pd
mkdir -p $R/$OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
for prog in "tt_p4:p4:0" "tt_pd:pd:0" "nt_pd:pd:1"; do
  name=${prog%%:*}; rest=${prog#*:}; kn=${rest%%:*}; nt=${rest#*:}
  i=0
  for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
             "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD" \
             "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    PMC_KERNEL=$kn PMC_NT=$nt timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/$OUT/${name}_p$i -o run -- python3 $R/scripts/wgrad_pmc_driver.py > $R/$OUT/${name}_p$i.log 2>&1 || { echo "$name pass $i failed"; tail -5 $R/$OUT/${name}_p$i.log; exit 1; }
    tail -1 $R/$OUT/${name}_p$i.log
  done
done
