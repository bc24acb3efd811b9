#!/bin/bash
# Interleaved bench A/B of the verification partial pass: the in-tree library (one shift per chunk,
# plain block sums) vs trustworthy_dl/_native_ab (the previous per-lane-shift + fp64 Chan merge
# build of csrc/stats.hip, everything else identical).  3 rounds, stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && mkdir -p gpurun_out/gpab
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in 1 2 3; do
  for f in old new; do
    if [ $f = old ]; then export TDL_NATIVE_LIB=$R/trustworthy_dl/_native_ab/libtdl_kernels.so; else unset TDL_NATIVE_LIB; fi
    timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 > gpurun_out/gpab/${f}_$i.log 2>&1
    rc=$?; echo "$f round $i rc=$rc $(tail -1 gpurun_out/gpab/${f}_$i.log | cut -c1-110)"; [ $rc -ne 0 ] && exit $rc
  done
done
unset TDL_NATIVE_LIB
cd /tmp && export TMPDIR=/tmp && export TDL_SERIALIZE_STREAMS=1 TDL_NATIVE_LIB=$R/trustworthy_dl/_native_ab/libtdl_kernels.so
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/gpab/prof_ser_old -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 > $R/gpurun_out/gpab/prof_ser_old.log 2>&1
rc=$?; echo "prof serialized old rc=$rc"
exit $rc
