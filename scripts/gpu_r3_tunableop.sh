#!/bin/bash
# hipBLASLt solution selection for the plain library GEMMs of the GPT-2-medium step (PyTorch
# TunableOp): tune once (every candidate solution timed per shape, results CSV), then an interleaved
# bench A/B: default heuristic vs the tuned file (tuning off).  Each GPU step time-limited.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
rm -f $R/gpurun_out/tunableop_gpt2m*.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
PYTORCH_TUNABLEOP_FILENAME=$R/gpurun_out/tunableop_gpt2m%d.csv \
PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=60 PYTORCH_TUNABLEOP_MAX_TUNING_ITERATIONS=30 \
  timeout -k 10 700 python -u bench.py --steps 1 --warmup 1 > $R/gpurun_out/tune.log 2>&1
rc=$?; echo "tune rc=$rc"; ls $R/gpurun_out/tunableop_gpt2m*.csv; [ $rc -ne 0 ] && { tail -5 $R/gpurun_out/tune.log; exit $rc; }
F=$(ls $R/gpurun_out/tunableop_gpt2m*.csv | head -1)
for i in 1 2 3; do
  PYTORCH_TUNABLEOP_ENABLED=0 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > $R/gpurun_out/ab_tune_off_$i.log 2>&1
  rc=$?; echo "off $i rc=$rc $(tail -1 $R/gpurun_out/ab_tune_off_$i.log | cut -c1-120)"; [ $rc -ne 0 ] && exit $rc
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$F \
    timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > $R/gpurun_out/ab_tune_on_$i.log 2>&1
  rc=$?; echo "on  $i rc=$rc $(tail -1 $R/gpurun_out/ab_tune_on_$i.log | cut -c1-120)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
