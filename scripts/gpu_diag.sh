#!/bin/bash
# Run each diagnostic case in its own process with its own timeout; stop at the first failure.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
export AMD_SERIALIZE_KERNEL=3
LOG=gpurun_out/diag.log
: > $LOG
for c in ${CASES:-fwd dgrad wgrad_f32_beta1 bias bgrada gelu_aux_bias linear_t attn_fwd attn_bwd}; do
  echo "== $c" >> $LOG
  timeout -k 10 240 python -u scripts/diag_gpu.py $c >> $LOG 2>&1
  rc=$?
  echo "rc=$rc" >> $LOG
  if [ $rc -ne 0 ]; then echo "STOP at $c rc=$rc"; cat $LOG; exit $rc; fi
done
cat $LOG
