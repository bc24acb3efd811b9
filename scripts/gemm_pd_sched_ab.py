#!/usr/bin/env python3
"""Schedule variants of the LDS-DMA persistent GEMM (csrc/gemm.hip gemm_pd, TDL_PD_SCHED) against
hipBLASLt and the ping-pong kernel on the GPT-2-medium forward / input-gradient products at 64k
tokens: interleaved rounds in one process, uniform random operands, every variant checked against
fp32 first.  One JSON line per product.
    python scripts/gemm_pd_sched_ab.py [--variants 0,1,2,3,4]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import gemm  # noqa: E402


def timer(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2,3,4")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--groups", default="", help="extra grouped tile orders for pd (TDL_GEMM_GROUPM)")
    args = ap.parse_args()
    M, C = 65536, 1024
    prods = [("qkv_fwd", C, 3 * C), ("o_fwd", C, C), ("fc_fwd", C, 4 * C), ("proj_fwd", 4 * C, C),
             ("qkv_dgrad", 3 * C, C)]
    os.environ["TDL_GEMM_GROUPM"] = "0"
    for name, K, N in prods:
        if args.only and name not in args.only.split(","):
            continue
        torch.manual_seed(1)
        a = ((torch.rand(M, K, device="cuda") * 2 - 1)).bfloat16()
        b = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16().t()
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        fns = {"lib": lambda: torch.mm(a, b, out=out),
               "pp": lambda: gemm._launch(a, b, out, N, "none", kernel="pp")}
        for v in args.variants.split(","):
            def f(v=v):
                os.environ["TDL_PD_SCHED"] = v
                os.environ.pop("TDL_PD_X4", None)
                gemm._launch(a, b, out, N, "none", kernel="pd")
            fns["pd" + v] = f

        def f_nox4():   # default schedule, per-tile-row stores instead of the 16-byte epilogue
            os.environ["TDL_PD_SCHED"] = "0"
            os.environ["TDL_PD_X4"] = "0"
            gemm._launch(a, b, out, N, "none", kernel="pd")
        fns["pd0_nox4"] = f_nox4
        for g in [x for x in args.groups.split(",") if x]:
            def f_g(g=g):   # default schedule and epilogue, grouped tile order
                os.environ["TDL_PD_SCHED"] = "0"
                os.environ.pop("TDL_PD_X4", None)
                os.environ["TDL_GEMM_GROUPM"] = g
                gemm._launch(a, b, out, N, "none", kernel="pd")
                os.environ["TDL_GEMM_GROUPM"] = "0"
            fns["pd0_g" + g] = f_g
        ref = a.float() @ b.float()
        bad = {}
        for k, f in fns.items():
            out.fill_(float("nan"))
            f()
            err = float((out.float() - ref).abs().max() / ref.abs().max())
            if not err < 0.02:
                bad[k] = err
        del ref
        times = {k: [] for k in fns}
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        for _ in range(args.rounds):
            for k, f in fns.items():
                times[k].append(timer(f, args.iters))
        flops = 2.0 * M * K * N
        res = {"product": name, "M": M, "K": K, "N": N, "bad": bad}
        for k, v in times.items():
            t = statistics.median(v)
            res[k + "_us"] = round(t * 1e6, 1)
            res[k + "_tf"] = round(flops / t / 1e12, 1)
        print(json.dumps(res), flush=True)
    os.environ.pop("TDL_PD_SCHED", None)
    os.environ.pop("TDL_PD_X4", None)


if __name__ == "__main__":
    main()
