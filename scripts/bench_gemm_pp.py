#!/usr/bin/env python3
"""Ping-pong native GEMM (tdl_gemm variant 20) vs the 8-wave kernel (variant 0) vs hipBLASLt
(torch.mm) on the GPT-2-medium NT products at 32k tokens, interleaved rounds in one process
(cdna_hip_programming.md rule 24), uniform random [-1, 1) operands (rule 25).  Correctness first:
ragged shapes and the fused epilogues against fp32 torch."""
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


def relerr(x, ref):
    return float((x.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-12))


def check(dev, variants):
    torch.manual_seed(0)
    out = []
    for (M, K, N) in [(1000, 128, 200), (256, 192, 256), (4104, 1024, 1032), (32768, 1024, 1024),
                      (8200, 512, 8200)]:  # last: > 1 tile per workgroup of the persistent form, ragged
        a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        bt = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
        bias = (torch.rand(N, device=dev) - 0.5).bfloat16()
        pre_ref = a.float() @ bt.float().t() + bias.float()
        gelu_ref = torch.nn.functional.gelu(pre_ref, approximate="tanh")
        for v in variants:
            gemm.VARIANT = v
            y = gemm.matmul(a, bt.t(), bias=bias)
            aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
            g = gemm.matmul(a, bt.t(), bias=bias, epi="gelu", aux=aux)
            acc = torch.zeros(M, N, dtype=torch.float32, device=dev)
            gemm._launch(a, bt.t(), acc, N, "f32acc")
            r = {"M": M, "K": K, "N": N, "variant": v, "bias": relerr(y, pre_ref), "gelu": relerr(g, gelu_ref),
                 "gelu_aux": relerr(aux, pre_ref), "f32acc": relerr(acc, pre_ref - bias.float())}
            out.append(r)
            print(json.dumps(r), flush=True)
        gemm.VARIANT = 0
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,20")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--no-check", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    vs = [int(v) for v in args.variants.split(",")]
    if not args.no_check:
        res = check(dev, vs)
        bad = [r for r in res if max(r["bias"], r["gelu"], r["gelu_aux"], r["f32acc"]) > 0.02]
        if bad:
            print(json.dumps({"check": "FAILED", "bad": bad}), flush=True)
            sys.exit(1)
    M = 32768
    shapes = [("fc_fwd|proj_dgrad", 1024, 4096), ("proj_fwd|fc_dgrad", 4096, 1024), ("qkv_fwd", 1024, 3072),
              ("o_fwd|o_dgrad", 1024, 1024), ("qkv_dgrad", 3072, 1024)]
    for name, K, N in shapes:
        a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        bt = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
        fns = {v: (lambda v=v: (setattr(gemm, "VARIANT", v), gemm.matmul(a, bt.t()))) for v in vs}
        fns[-1] = lambda: torch.mm(a, bt.t())
        times = {k: [] for k in fns}
        for f in fns.values():
            f()
        for _ in range(args.rounds):
            for k, f in fns.items():
                times[k].append(timer(f, args.iters))
        gemm.VARIANT = 0
        fl = 2.0 * M * K * N
        row = {"shape": name, "M": M, "K": K, "N": N, "hipblaslt_tf": round(fl / statistics.median(times[-1]) / 1e12, 1)}
        for v in vs:
            tf = fl / statistics.median(times[v]) / 1e12
            row[f"v{v}_tf"] = round(tf, 1)
            row[f"v{v}_vs_lib"] = round(tf / row["hipblaslt_tf"], 3)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
