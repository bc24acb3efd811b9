#!/bin/bash
# Register-resident cross-entropy kernel: GPU numerics, then N=1 bench A/B vs the two-pass kernel.
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -k "xent or lm_head" > gpurun_out/xent_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/xent_pytest.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in 0 1; do
    TDL_XENT_REG=$v timeout -k 10 300 python -u bench.py --steps 8 --warmup 3 > gpurun_out/xent_$v.$r.log 2>&1 || { tail -20 gpurun_out/xent_$v.$r.log; exit 1; }
    echo "xent_reg=$v run $r: $(grep metric gpurun_out/xent_$v.$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_v11 -o run -- python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/prof_v11.log 2>&1 || { tail -20 $R/gpurun_out/prof_v11.log; exit 1; }
f=$(find $R/gpurun_out/prof_v11 -name "*kernel_stats.csv" | head -1)
python3 $R/scripts/prof_summary.py "$f" 7 40 > $R/gpurun_out/prof_v11_summary.txt
head -30 $R/gpurun_out/prof_v11_summary.txt
