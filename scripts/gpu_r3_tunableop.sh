#!/bin/bash
# hipBLASLt / rocBLAS solution selection for the plain library GEMMs of the GPT-2-medium step
# (PyTorch TunableOp): tune the shapes the committed results file does not hold yet (every candidate
# solution timed per shape), then an interleaved bench A/B: default heuristic vs the tuned file
# (lookup only).  Each GPU step time-limited; a heartbeat file keeps the long tuning step visible.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
SRC=$R/trustworthy_dl/tuning/tunableop_gpt2m_mi355x.csv
F=$R/gpurun_out/tunableop_gpt2m0.csv
[ -f $SRC ] && cp $SRC $F
( while true; do sleep 30; date +%T >> $R/gpurun_out/tune_tick.log; done ) &
HB=$!
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
PYTORCH_TUNABLEOP_FILENAME=$R/gpurun_out/tunableop_gpt2m%d.csv \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=60 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=30 \
  timeout -k 10 800 python -u bench.py --steps 1 --warmup 1 > $R/gpurun_out/tune.log 2>&1
rc=$?; kill $HB; echo "tune rc=$rc"; wc -l $F; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/tune.log; exit $rc; }
for i in 1 2 3; do
  TDL_TUNED_GEMMS=0 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > $R/gpurun_out/ab_tune_off_$i.log 2>&1
  rc=$?; echo "off $i rc=$rc $(tail -1 $R/gpurun_out/ab_tune_off_$i.log | cut -c1-120)"; [ $rc -ne 0 ] && exit $rc
  TDL_TUNED_GEMMS=$F timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > $R/gpurun_out/ab_tune_on_$i.log 2>&1
  rc=$?; echo "on  $i rc=$rc $(tail -1 $R/gpurun_out/ab_tune_on_$i.log | cut -c1-120)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
