#!/bin/bash
# PMC passes over the weight-gradient kernel (scripts/wgrad_pmc_driver.py), one counter group per run
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${PMC_OUT:-pmc_wgrad}
mkdir -p $R/gpurun_out/$OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 120 python3 $R/scripts/wgrad_pmc_driver.py > $R/gpurun_out/$OUT/plain.log 2>&1 || { echo "plain run failed"; tail -5 $R/gpurun_out/$OUT/plain.log; exit 1; }
cat $R/gpurun_out/$OUT/plain.log
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM_RD" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/$OUT/p$i -o run -- python3 $R/scripts/wgrad_pmc_driver.py > $R/gpurun_out/$OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/$OUT/p$i.log; exit 1; }
done
ls -R $R/gpurun_out/$OUT | head -30
