#!/bin/bash
# PMC pass (SQ group: MFMA busy, waits) over the qkv weight gradient alone on gemm_pd (split 16,
# three rounds) and the qkv + o pair from one grouped launch (split 4, one round), 64k tokens.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=gpurun_out/pmc_wgrad_grouped
mkdir -p $R/$OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
for prog in "tt_pd:pd" "grouped:grouped"; do
  name=${prog%%:*}; kn=${prog#*:}
  set="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
  PMC_KERNEL=$kn timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $R/$OUT/${name}_p1 -o run -- python3 $R/scripts/wgrad_pmc_driver.py > $R/$OUT/${name}_p1.log 2>&1 || { echo "$name failed"; tail -5 $R/$OUT/${name}_p1.log; exit 1; }
  tail -1 $R/$OUT/${name}_p1.log
done
cd $R && python3 scripts/pmc_summary.py $OUT
