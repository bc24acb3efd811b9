#!/bin/bash
# PMC counter passes over the GEMM driver (one pass per counter group, no tracing domains).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=${PMC_OUT:-pmc_gemm}
mkdir -p $R/gpurun_out/$OUT
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  for prog in ${PROGS:-gemm_only}; do
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/$OUT/${prog}_p$i -o run -- python3 $R/scripts/$prog.py > $R/gpurun_out/$OUT/${prog}_p$i.log 2>&1 || { echo "pass $i $prog failed"; tail -5 $R/gpurun_out/$OUT/${prog}_p$i.log; exit 1; }
  done
done
ls $R/gpurun_out/$OUT
