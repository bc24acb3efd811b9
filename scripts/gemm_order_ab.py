#!/usr/bin/env python3
"""Tile-order A/B for the native GEMMs (csrc/gemm.hip TDL_GEMM_GROUPM) against hipBLASLt on the
GPT-2-medium forward / input-gradient products at 64k tokens: interleaved rounds in one process
(cdna_hip_programming.md rule 24), uniform random operands (rule 25).  One JSON line per product.
    python scripts/gemm_order_ab.py [--groups 0,4,8,16] [--kernels pp] [--epi none,gelu]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import gemm  # noqa: E402


def rnd(*shape, scale=1.0):
    return ((torch.rand(*shape, device="cuda") * 2 - 1) * scale).bfloat16()


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
    ap.add_argument("--groups", default="0,4,8,16")
    ap.add_argument("--kernels", default="pp")
    ap.add_argument("--epi", default="none")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    M, C = args.tokens, 1024
    prods = [("qkv_fwd", C, 3 * C), ("o_fwd", C, C), ("fc_fwd", C, 4 * C), ("proj_fwd", 4 * C, C),
             ("qkv_dgrad", 3 * C, C)]
    groups = [int(g) for g in args.groups.split(",")]
    for name, K, N in prods:
        if args.only and name not in args.only.split(","):
            continue
        torch.manual_seed(1)
        a = rnd(M, K)
        b = rnd(N, K, scale=0.05).t()
        bias = rnd(N, scale=0.5)
        out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        aux = torch.empty_like(out)
        cs = torch.zeros(N, device="cuda")
        ref = None
        fns = {"lib": lambda: torch.mm(a, b, out=out)}
        for epi in args.epi.split(","):
            for kn in args.kernels.split(","):
                for g in groups:
                    def f(kn=kn, g=g, epi=epi):
                        os.environ["TDL_GEMM_GROUPM"] = str(g)
                        gemm.KERNEL = kn
                        if epi == "none":
                            gemm.matmul(a, b, out=out)
                        elif epi == "bias":
                            gemm.matmul(a, b, bias=bias, out=out)
                        elif epi == "gelu":
                            gemm.matmul(a, b, bias=bias, out=out, epi="gelu", aux=aux)
                        elif epi == "dgelu":
                            gemm.matmul(a, b, out=out, epi="dgelu", aux=aux, colsum=cs)
                    fns[f"{kn}_{epi}_g{g}"] = f
        # correctness of every order on the plain product
        ref = (a.float() @ b.float())
        bad = {}
        for g in groups:
            os.environ["TDL_GEMM_GROUPM"] = str(g)
            for kn in args.kernels.split(","):
                gemm.KERNEL = kn
                y = gemm.matmul(a, b)
                err = float((y.float() - ref).abs().max() / ref.abs().max())
                if err > 0.02:
                    bad[f"{kn}_g{g}"] = err
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
    os.environ.pop("TDL_GEMM_GROUPM", None)


if __name__ == "__main__":
    main()
