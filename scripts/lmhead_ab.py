#!/usr/bin/env python3
"""LM-head GEMMs at the N = 1 bench shape (64 x 1024 tokens, vocab padded to 50304), interleaved:
  fwd : logits [N, Vp] = x [N, 1024] @ W^T    library (torch.mm) vs gemm_pd (NT: W is [Vp][1024])
  dX  : dx [N, 1024] = dL [N, Vp] @ W         library vs gemm_pd on a [1024][Vp] copy of W (NT)
One JSON line per (product, kernel): median us, TF/s, max relative error vs fp32.

    python scripts/lmhead_ab.py --out gpurun_out/r6_lmhead_ab.jsonl
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import gemm  # noqa: E402


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def pd(a, b, out):
    old = gemm.KERNEL
    gemm.KERNEL = "pd"
    try:
        return gemm.matmul(a, b, out=out)
    finally:
        gemm.KERNEL = old


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=65536)
    ap.add_argument("--Vp", type=int, default=50304)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--groups", default="")
    ap.add_argument("--out", default="gpurun_out/r6_lmhead_ab.jsonl")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    f = open(a.out, "a")
    N, Vp, C = a.N, a.Vp, 1024
    torch.manual_seed(0)
    x = (torch.rand(N, C, device="cuda") * 2 - 1).bfloat16()
    w = ((torch.rand(Vp, C, device="cuda") * 2 - 1) * 0.05).bfloat16()
    wt = w.t().contiguous()
    logits = torch.empty(N, Vp, dtype=torch.bfloat16, device="cuda")
    dl = ((torch.rand(N, Vp, device="cuda") * 2 - 1) * 1e-3).bfloat16()
    dx = torch.empty(N, C, dtype=torch.bfloat16, device="cuda")
    variants = {
        "fwd_lib": lambda: torch.mm(x, w.t(), out=logits),
        "fwd_pd": lambda: pd(x, w.t(), logits),
        "dx_lib": lambda: torch.mm(dl, w, out=dx),
        "dx_pd": lambda: pd(dl, wt.t(), dx),
    }
    for g in [s for s in a.groups.split(",") if s]:
        def run(g=g):
            os.environ["TDL_GEMM_GROUPM"] = g
            pd(x, w.t(), logits)
            os.environ.pop("TDL_GEMM_GROUPM", None)
        variants[f"fwd_pd_g{g}"] = run
    flops = {"fwd": 2.0 * N * Vp * C, "dx": 2.0 * N * Vp * C}
    # correctness on a row block (fp32 reference)
    errs = {}
    rows = slice(0, 2048)
    for k, fn in variants.items():
        fn()
        torch.cuda.synchronize()
        if k.startswith("fwd"):
            ref = x[rows].float() @ w.float().t()
            got = logits[rows].float()
        else:
            ref = dl[rows].float() @ w.float()
            got = dx[rows].float()
        errs[k] = float((got - ref).abs().max() / ref.abs().max())
    times = {k: [] for k in variants}
    for _ in range(a.rounds):
        for k, fn in variants.items():
            times[k].append(timed(fn, a.iters))
    for k, ts in times.items():
        us = statistics.median(ts)
        rec = {"product": k.split("_")[0], "variant": k, "N": N, "Vp": Vp, "us": round(us, 1),
               "tflops": round(flops[k.split("_")[0]] / us / 1e6, 1), "spread_us": round(max(ts) - min(ts), 1),
               "relerr": errs[k]}
        print(json.dumps(rec), flush=True)
        f.write(json.dumps(rec) + "\n")
    f.close()


if __name__ == "__main__":
    main()
