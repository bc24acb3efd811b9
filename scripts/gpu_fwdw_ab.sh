#!/bin/bash
# Forward-layout weight copies: GPU tests, then N=1 bench A/B (interleaved) with TDL_FWD_WEIGHT_T=1/0.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_fwd_weight_gpu.py tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/fwdw_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/fwdw_pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in 1 0; do
    TDL_FWD_WEIGHT_T=$v timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 ${BENCH_ARGS} > gpurun_out/fwdw_$v.$r.log 2>&1 || { tail -20 gpurun_out/fwdw_$v.$r.log; exit 1; }
    echo "fwd_weight_t=$v run $r: $(grep metric gpurun_out/fwdw_$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
