#!/usr/bin/env python3
"""Tied LM-head weight gradient at the bench shape (dW [50304, 1024] += dlogits^T x, 64k tokens):
gemm_pd at the cost model's split and at fixed splits vs the library GEMM with an fp32 output
(torch.mm(out_dtype=float32)) plus the accumulate, interleaved rounds, median us.

    python scripts/lm_wgrad_ab.py --out gpurun_out/r6_lm_wgrad_ab.jsonl
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--groups", default="")
    ap.add_argument("--splits", default="1,2,3,4,6,8")
    ap.add_argument("--lib", type=int, default=1)
    ap.add_argument("--out", default="gpurun_out/r6_lm_wgrad_ab.jsonl")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    f = open(a.out, "a")
    T, V, C = a.tokens, 50304, 1024
    torch.manual_seed(0)
    dl = ((torch.rand(T, V, device="cuda") * 2 - 1) * 0.01).bfloat16()
    x = (torch.rand(T, C, device="cuda") * 2 - 1).bfloat16()
    acc = torch.zeros(V, C, device="cuda")
    variants = {"pd_model": lambda: gemm.matmul_f32_acc(acc, dl.t(), x, kernel="pd")}
    for s in (int(v) for v in a.splits.split(",") if v):
        variants[f"pd_s{s}"] = lambda s=s: gemm.matmul_f32_acc(acc, dl.t(), x, split=s, kernel="pd")
    if a.lib:
        variants["lib_f32"] = lambda: acc.add_(torch.mm(dl.t(), x, out_dtype=torch.float32))
    for g in (v for v in a.groups.split(",") if v):   # tile orders (TDL_GEMM_GROUPM, read per launch) at the model's split
        def run(g=g):
            os.environ["TDL_GEMM_GROUPM"] = g
            gemm.matmul_f32_acc(acc, dl.t(), x, kernel="pd")
            os.environ.pop("TDL_GEMM_GROUPM", None)
        variants[f"pd_g{g}"] = run
    times = {k: [] for k in variants}
    for fn in variants.values():
        fn()
    for _ in range(a.rounds):
        for k, fn in variants.items():
            times[k].append(timed(fn, a.iters))
    for k, ts in times.items():
        us = statistics.median(ts)
        rec = {"tokens": T, "variant": k, "us": round(us, 1), "tflops": round(2.0 * T * V * C / us / 1e6, 1),
               "spread_us": round(max(ts) - min(ts), 1), "model_split": gemm.wgrad_split(T, V, C)}
        print(json.dumps(rec), flush=True)
        f.write(json.dumps(rec) + "\n")
    f.close()


if __name__ == "__main__":
    main()
