#!/bin/bash
# gemm_pd (4-wave persistent, LDS-DMA on the library's schedule): numerics (every NT test with pd),
# then its schedule variants against hipBLASLt and the ping-pong kernel (interleaved, one process)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -k "pd" -x -q --timeout 120 --timeout-method thread > gpurun_out/gemm_pd_t.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gemm_pd_t.log; exit 1; }
tail -2 gpurun_out/gemm_pd_t.log
timeout -k 10 400 python -u scripts/gemm_pd_sched_ab.py ${PD_ARGS} > gpurun_out/gemm_pd_ab.jsonl 2>&1 || { echo "ab failed"; tail -20 gpurun_out/gemm_pd_ab.jsonl; exit 1; }
python3 - <<'PY'
import json
for l in open("gpurun_out/gemm_pd_ab.jsonl"):
    if not l.startswith("{"): continue
    r = json.loads(l)
    print(r["product"], "bad", r["bad"], {k[:-3]: v for k, v in r.items() if k.endswith("_tf")})
PY
