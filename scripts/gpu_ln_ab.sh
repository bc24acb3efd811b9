#!/bin/bash
# LayerNorm backward rows-per-wave A/B: numerics with the default choice (8 rows per wave for the
# four-set variant, 2 otherwise), N=1 bench interleaved default ("0") vs forced 2, then rocprof stats.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_block.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ln_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/ln_pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in 0 2; do
    TDL_LN_RPW=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/ln_$v.$r.log 2>&1 || { tail -20 gpurun_out/ln_$v.$r.log; exit 1; }
    echo "ln_rpw=$v run $r: $(grep metric gpurun_out/ln_$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_v17 -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof_v17.log 2>&1 || { tail -20 $R/gpurun_out/prof_v17.log; exit 1; }
f=$(find $R/gpurun_out/prof_v17 -name "*kernel_stats.csv" | head -1)
python3 $R/scripts/prof_summary.py "$f" 7 40 > $R/gpurun_out/prof_v17_summary.txt
grep -E "total|ln_bwd|colsum" $R/gpurun_out/prof_v17_summary.txt
