#!/bin/bash
# Step-tail host syncs removed (scalar writes via fill_, cached index tensors) + per-segment
# workgroup merge: pytest -m gpu, then an interleaved bench A/B against the previous tree (ab_old/,
# a git worktree of the previous commit running on the same native library), then a HIP API +
# kernel trace of the new tree.  Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/sf
export HSA_ENABLE_IPC_MODE_LEGACY=0
[ -n "$SKIP_PYTEST" ] || timeout -k 10 600 python -u -m pytest tests/ -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/sf/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do
  for f in old new; do
    if [ $f = old ]; then d=$R/ab_old; export TDL_NATIVE_LIB=$R/trustworthy_dl/_native/libtdl_kernels.so; else d=$R; unset TDL_NATIVE_LIB; fi
    (cd $d && timeout -k 10 200 python -u bench.py --steps 10 --warmup 3) > gpurun_out/sf/${f}_$i.log 2>&1
    rc=$?; echo "$f round $i rc=$rc $(tail -1 gpurun_out/sf/${f}_$i.log | cut -c1-110)"; [ $rc -ne 0 ] && exit $rc
  done
done
unset TDL_NATIVE_LIB
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d $R/gpurun_out/sf/ht -o run -- \
  python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/sf/ht_bench.log 2>&1
rc=$?; echo "trace rc=$rc"
exit $rc
