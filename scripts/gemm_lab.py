#!/usr/bin/env python3
"""Native GEMM kernels (csrc/gemm.hip: p4 = persistent 4-wave, pp = staggered ping-pong) against
hipBLASLt (torch) on every GEMM product of a GPT-2-medium step at 64k tokens, plus fp32 checks.

Correctness first (ragged shapes, all four operand layouts, every epilogue, vs fp32 torch); then
interleaved timing rounds in one process (cdna_hip_programming.md rule 24) on uniform random
operands (rule 25).  One JSON line per product: TFLOP/s per kernel, ratio to the library.
    python scripts/gemm_lab.py [--kernels p4,pp] [--rounds 5] [--only fwd,dgrad,wgrad,lmhead]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import gemm  # noqa: E402
from trustworthy_dl.ops import layers  # noqa: E402


def relerr(x, ref):
    return float((x.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-12))


def rnd(*shape, scale=1.0, dev="cuda"):
    return ((torch.rand(*shape, device=dev) * 2 - 1) * scale).bfloat16()


def check(kernels, dev):
    """every layout x epilogue at ragged shapes; returns the failures"""
    torch.manual_seed(0)
    bad = []
    for (M, K, N) in [(1000, 128, 200), (256, 192, 264), (4104, 1024, 1032), (2048, 4096, 1024), (8200, 512, 8200)]:
        for ta in (0, 1):
            for tb in (0, 1):
                a_ = rnd(M, K) if not ta else rnd(K, M).t()
                b_ = rnd(K, N, scale=0.05) if tb else rnd(N, K, scale=0.05).t()
                bias = rnd(N, scale=0.5)
                ref = a_.float() @ b_.float()
                for kn in kernels:
                    gemm.KERNEL = kn
                    r = {"M": M, "K": K, "N": N, "ta": ta, "tb": tb, "kernel": kn}
                    try:
                        y = gemm.matmul(a_, b_, bias=bias)
                        r["bias"] = relerr(y, ref + bias.float())
                        aux = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
                        g = gemm.matmul(a_, b_, bias=bias, epi="gelu", aux=aux)
                        r["gelu"] = relerr(g, torch.nn.functional.gelu(ref + bias.float(), approximate="tanh"))
                        c = rnd(M, N)
                        c0 = c.float().clone()
                        gemm.matmul(a_, b_, out=c, epi="resadd")
                        r["resadd"] = relerr(c, c0 + ref)
                        acc = torch.randn(M, N, device=dev)
                        acc0 = acc.clone()
                        gemm.matmul_f32_acc(acc, a_, b_, split=1)
                        r["f32acc"] = relerr(acc, acc0 + ref)
                        if kn != "pp" or K // gemm.effective_split(K, 4) >= 128:
                            acc = torch.zeros(M, N, device=dev)
                            gemm.matmul_f32_acc(acc, a_, b_, split=4, mode="atomic")
                            r["f32atomic4"] = relerr(acc, ref)
                        if kn != "pp" or K // gemm.effective_split(K, 2) >= 128:
                            acc = torch.zeros(M, N, device=dev)
                            gemm.matmul_f32_acc(acc, a_, b_, split=2, mode="slab")
                            r["f32slab2"] = relerr(acc, ref)
                        if not ta:
                            pre = rnd(M, N, scale=2.0)
                            cs = torch.zeros(N, device=dev)
                            d = gemm.matmul(a_, b_, epi="dgelu", aux=pre, colsum=cs)
                            u = pre.float().requires_grad_(True)
                            gg, = torch.autograd.grad(torch.nn.functional.gelu(u, approximate="tanh"), u, ref)
                            r["dgelu"] = relerr(d, gg)
                            r["colsum"] = relerr(cs, gg.sum(0))
                    except Exception as e:  # noqa: BLE001
                        r["error"] = repr(e)
                    torch.cuda.synchronize()
                    vals = [v for k, v in r.items() if isinstance(v, float)]
                    worst = float("inf") if any(v != v for v in vals) else max(vals + [0.0])
                    r["worst"] = worst
                    if worst > 0.02 or "error" in r:
                        bad.append(r)
                    print(json.dumps(r), flush=True)
    return bad


def products(M=65536, C=1024, V=50304):
    """(name, a_shape_storage, b_shape_storage, ta, tb, epi-kind)"""
    P = []
    for name, K, N in [("qkv_fwd", C, 3 * C), ("o_fwd", C, C), ("fc_fwd", C, 4 * C), ("proj_fwd", 4 * C, C)]:
        P.append((name, M, K, N, 0, 0, "fwd"))
    for name, K, N in [("proj_dgrad", C, 4 * C), ("fc_dgrad", 4 * C, C), ("o_dgrad", C, C), ("qkv_dgrad", 3 * C, C)]:
        P.append((name, M, K, N, 0, 0, "fwd"))
    for name, Kin, Nout in [("qkv_wgrad", C, 3 * C), ("o_wgrad", C, C), ("fc_wgrad", C, 4 * C), ("proj_wgrad", 4 * C, C)]:
        P.append((name, Kin, M, Nout, 1, 1, "wgrad"))
    P.append(("lmhead_fwd", M, C, V, 0, 0, "fwd"))
    P.append(("lmhead_dx", M, V, C, 0, 1, "fwd"))
    P.append(("lmhead_dw", V, M, C, 1, 1, "wgrad"))
    return P


def make_operands(Mg, K, N, ta, tb, dev):
    a = rnd(K, Mg).t() if ta else rnd(Mg, K)
    b = rnd(K, N, scale=0.05) if tb else rnd(N, K, scale=0.05).t()
    return a, b


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
    ap.add_argument("--kernels", default="p4,pp")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--only", default="")
    ap.add_argument("--splits", default="", help="wgrad split-K factors to try for p4, e.g. 4,8,16")
    ap.add_argument("--no-check", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    kernels = [k for k in args.kernels.split(",") if k]
    if not args.no_check:
        bad = check(kernels, dev)
        print(json.dumps({"check": "FAILED" if bad else "ok", "n_bad": len(bad)}), flush=True)
        if bad:
            sys.exit(1)
    only = set(x for x in args.only.split(",") if x)
    for name, Mg, K, N, ta, tb, kind in products(M=args.tokens):
        if only and not any(o in name for o in only):
            continue
        torch.manual_seed(1)
        a, b = make_operands(Mg, K, N, ta, tb, dev)
        flops = 2.0 * Mg * K * N
        fns = {}
        if kind == "fwd":
            out = torch.empty(Mg, N, dtype=torch.bfloat16, device=dev)
            fns["lib"] = lambda: torch.mm(a, b, out=out)
            for kn in kernels:
                if kn == "pp" and (ta or tb):
                    continue
                fns[kn] = (lambda kn=kn: (setattr(gemm, "KERNEL", kn), gemm.matmul(a, b, out=out)))
        else:
            acc = torch.zeros(Mg, N, dtype=torch.float32, device=dev)
            fns["lib"] = lambda: layers.wgrad_acc(acc, a, b)
            splits = [int(x) for x in args.splits.split(",") if x] or [gemm.wgrad_split(K, Mg, N)]
            for kn in kernels:
                for S in splits:
                    for mode in ("atomic", "slab"):
                        fns[f"{kn}_s{S}_{mode}"] = (lambda kn=kn, S=S, mode=mode: (
                            setattr(gemm, "KERNEL", kn), gemm.matmul_f32_acc(acc, a, b, split=S, mode=mode)))
        times = {k: [] for k in fns}
        for k, f in fns.items():  # warm-up
            f()
        torch.cuda.synchronize()
        for _ in range(args.rounds):
            for k, f in fns.items():
                times[k].append(timer(f, args.iters))
        med = {k: statistics.median(v) for k, v in times.items()}
        res = {"product": name, "M": Mg, "K": K, "N": N, "ta": ta, "tb": tb}
        for k, t in med.items():
            res[k + "_us"] = round(t * 1e6, 1)
            res[k + "_tf"] = round(flops / t / 1e12, 1)
        best = min((t, k) for k, t in med.items() if k != "lib")
        res["best"] = best[1]
        res["best_vs_lib"] = round(med["lib"] / best[0], 3)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
