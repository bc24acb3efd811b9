#!/usr/bin/env python3
"""Tile-order / split A/B for the persistent weight-gradient kernel (gemm_p4, fp32 main_grad +=
x^T dy with split-K slabs + reduce) on the four GPT-2-medium block weight gradients at 64k tokens:
TDL_GEMM_GROUPM (0 = row-major, G = groups of G tile rows, tile column slowest) x split, interleaved
rounds in one process, uniform random operands.  One JSON line per product.
    python scripts/wgrad_order_ab.py [--groups 0,2,4,8] [--splits auto,8,16]
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
    ap.add_argument("--groups", default="0,2,4,8")
    ap.add_argument("--splits", default="auto")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--only", default="")
    ap.add_argument("--kernels", default="p4", help="weight-gradient kernels to compare (p4, pd)")
    args = ap.parse_args()
    T, C = args.tokens, 1024
    prods = [("qkv_wgrad", C, 3 * C), ("o_wgrad", C, C), ("fc_wgrad", C, 4 * C), ("proj_wgrad", 4 * C, C)]
    groups = [int(g) for g in args.groups.split(",")]
    for name, cin, cout in prods:
        if args.only and name not in args.only.split(","):
            continue
        torch.manual_seed(1)
        x = ((torch.rand(T, cin, device="cuda") * 2 - 1)).bfloat16()
        dy = ((torch.rand(T, cout, device="cuda") * 2 - 1) * 0.05).bfloat16()
        acc = torch.zeros(cin, cout, dtype=torch.float32, device="cuda")
        auto = gemm.wgrad_split(T, cin, cout)
        splits = sorted({auto if s == "auto" else int(s) for s in args.splits.split(",")})
        fns = {}
        for kn in args.kernels.split(","):
            for sp in splits:
                for g in groups:
                    def f(g=g, sp=sp, kn=kn):
                        os.environ["TDL_GEMM_GROUPM"] = str(g)
                        gemm.matmul_f32_acc(acc, x.t(), dy, split=sp, kernel=kn)
                    fns[f"{kn}_s{sp}_g{g}"] = f
        # correctness of every variant: one accumulation from zero against fp32
        ref = x.float().t() @ dy.float()
        bad = {}
        for k, f in fns.items():
            acc.zero_()
            f()
            err = float((acc - ref).abs().max() / ref.abs().max())
            if err > 1e-3:
                bad[k] = err
        del ref
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        times = {k: [] for k in fns}
        for _ in range(args.rounds):
            for k, f in fns.items():
                times[k].append(timer(f, args.iters))
        flops = 2.0 * T * cin * cout
        res = {"product": name, "M": cin, "N": cout, "K": T, "auto_split": auto, "bad": bad}
        for k, v in times.items():
            t = statistics.median(v)
            res[k + "_us"] = round(t * 1e6, 1)
            res[k + "_tf"] = round(flops / t / 1e12, 1)
        print(json.dumps(res), flush=True)
    os.environ.pop("TDL_GEMM_GROUPM", None)


if __name__ == "__main__":
    main()
