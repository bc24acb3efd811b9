#!/usr/bin/env python3
"""In-kernel timeline of the native GEMMs (csrc/gemm.hip ``stamp``: s_memrealtime, 100 MHz, wave 0
of every workgroup): per-tile K-loop and epilogue time, start spread, against the kernel's event
time.  Diagnoses where the time between the MFMA bound and the measured time goes.
    python scripts/gemm_timeline.py [--kernels pp,p4,p4l] [--only qkv_fwd,fc_fwd]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import _lib, gemm  # noqa: E402

TICK_US = 0.01   # s_memrealtime: 100 MHz


def rnd(*shape, scale=1.0):
    return ((torch.rand(*shape, device="cuda") * 2 - 1) * scale).bfloat16()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", default="pp,p4,p4l")
    ap.add_argument("--only", default="qkv_fwd,fc_fwd,proj_fwd")
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--epi", default="none")
    args = ap.parse_args()
    M, C = args.tokens, 1024
    prods = {"qkv_fwd": (C, 3 * C), "o_fwd": (C, C), "fc_fwd": (C, 4 * C), "proj_fwd": (4 * C, C),
             "qkv_dgrad": (3 * C, C)}
    ts = torch.zeros(65536 * 64, dtype=torch.int64, device="cuda")
    for name in args.only.split(","):
        K, N = prods[name]
        a = rnd(M, K)
        b = rnd(N, K, scale=0.05).t()
        bias = rnd(N, scale=0.5)
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        aux = torch.empty_like(out)
        for kn in args.kernels.split(","):
            gemm.KERNEL = kn

            def run():
                if args.epi == "gelu":
                    gemm.matmul(a, b, bias=bias, out=out, epi="gelu", aux=aux)
                else:
                    gemm.matmul(a, b, out=out)
            for _ in range(3):
                run()
            ts.zero_()
            torch.cuda.synchronize()
            _lib.call("tdl_gemm_set_timestamps", ts.data_ptr())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            e1.synchronize()
            _lib.call("tdl_gemm_set_timestamps", None)
            ms = e0.elapsed_time(e1)
            t = ts.view(-1, 64).cpu()
            used = t[:, 0] > 0
            t = t[used]
            t0 = int(t[:, 0].min())
            res = {"product": name, "kernel": kn, "epi": args.epi, "event_us": round(ms * 1e3, 1), "workgroups": int(used.sum())}
            if kn in ("pp", "pr"):
                kl = ((t[:, 1] - t[:, 0]).float() * TICK_US)
                ep = ((t[:, 2] - t[:, 1]).float() * TICK_US)
                st = ((t[:, 0] - t0).float() * TICK_US)
                res.update({"kloop_us_med": round(float(kl.median()), 2), "kloop_us_p10": round(float(kl.quantile(0.1)), 2),
                            "kloop_us_p90": round(float(kl.quantile(0.9)), 2),
                            "epi_us_med": round(float(ep.median()), 2), "epi_us_p90": round(float(ep.quantile(0.9)), 2),
                            "span_us": round(float(((t[:, 2].max() - t0).float()) * TICK_US), 1),
                            "start_gap_us_med": None})
                # per-CU occupancy: sort starts; the gap between a workgroup's end and the next start
                # on the chip is the dispatch cost (approximate: one workgroup per CU)
                ends = sorted(int(x) for x in t[:, 2])
                starts = sorted(int(x) for x in t[:, 0])
                nwg = len(starts)
                gaps = [(starts[i] - ends[i - 256]) * TICK_US for i in range(256, nwg)]
                if gaps:
                    res["start_gap_us_med"] = round(statistics.median(gaps), 2)
            else:
                kls, eps = [], []
                for row in t.tolist():
                    prev = row[0]
                    for i in range(31):
                        k1, k2 = row[1 + 2 * i], row[2 + 2 * i]
                        if k1 == 0:
                            break
                        kls.append((k1 - prev) * TICK_US)
                        eps.append((k2 - k1) * TICK_US)
                        prev = k2
                res.update({"tiles": len(kls), "kloop_us_med": round(statistics.median(kls), 2),
                            "kloop_first_us_med": round(statistics.median([(r[1] - r[0]) * TICK_US for r in t.tolist()]), 2),
                            "epi_us_med": round(statistics.median(eps), 2),
                            "span_us": round(float(((t.max() - t0).float()) * TICK_US), 1)})
            flops = 2.0 * M * K * N
            res["tf"] = round(flops / (ms * 1e-3) / 1e12, 1)
            print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
