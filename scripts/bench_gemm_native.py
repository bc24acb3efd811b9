#!/usr/bin/env python3
"""Native MFMA GEMM (csrc/gemm.hip) vs torch.mm (hipBLASLt) on the GPT-2 block shapes.

For each shape and product (fwd / dgrad / wgrad) the native kernel is checked against an fp32
torch reference of the same bf16 inputs, then both are timed in interleaved rounds in one process
(cdna_hip_programming.md rule 24) on uniform random data.  One JSON line per (shape, product):
TFLOP/s median and min over rounds for ours and torch.

    python scripts/bench_gemm_native.py [--tokens 32768] [--rounds 5] [--iters 10] [--only qkv,o]
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


def timer(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def relerr(x, ref):
    return float((x.float() - ref).abs().max() / ref.abs().max().clamp(min=1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--products", default="fwd,fwd_nt,dgrad,wgrad,wgrad_atomic")
    ap.add_argument("--model", default="medium")
    ap.add_argument("--plain", action="store_true", help="also time a comparison variant of the native kernel")
    ap.add_argument("--plain-variant", type=int, default=10,
                    help="tdl_gemm variant id: 10 = 8-wave non-persistent, 11 = 4-wave persistent, 12 = no K rotation")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    C = 1024 if args.model == "medium" else 768
    shapes = [("qkv", C, 3 * C), ("o", C, C), ("fc", C, 4 * C), ("proj", 4 * C, C)]
    if args.only:
        shapes = [s for s in shapes if s[0] in args.only.split(",")]
    prods = args.products.split(",")
    M = args.tokens
    g = torch.Generator(device=dev).manual_seed(0)
    for name, K, N in shapes:
        x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(K, N, device=dev, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16)
        wt = w.t().contiguous()
        dy = (torch.rand(M, N, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        fl = 2.0 * M * K * N
        for prod in prods:
            if prod == "fwd":
                ours = lambda: gemm.matmul(x, w)
                ref_fn = lambda: torch.mm(x, w)
                ref = x.float() @ w.float()
            elif prod == "fwd_nt":
                ours = lambda: gemm.matmul(x, wt.t())
                ref_fn = lambda: torch.mm(x, wt.t())
                ref = x.float() @ w.float()
            elif prod == "dgrad":
                ours = lambda: gemm.matmul(dy, w.t())
                ref_fn = lambda: torch.mm(dy, w.t())
                ref = dy.float() @ w.float().t()
            elif prod in ("wgrad", "wgrad_atomic"):
                acc = torch.zeros(K, N, device=dev)
                mode = "atomic" if prod == "wgrad_atomic" else "slab"
                ours = lambda: gemm.matmul_f32_acc(acc, x.t(), dy, mode=mode)
                acc_t = torch.zeros(K, N, device=dev)
                ref_fn = lambda: layers.wgrad_acc(acc_t, x.t(), dy)
                ref = x.float().t() @ dy.float()
            else:
                continue
            # correctness (fresh accumulators for the fp32 products)
            if prod.startswith("wgrad"):
                acc.zero_()
                ours()
                err = relerr(acc, ref)
            else:
                err = relerr(ours(), ref)
            torch.cuda.synchronize()
            t_o, t_r, t_p = [], [], []
            ours(); ref_fn()
            for _ in range(args.rounds):
                t_o.append(timer(ours, args.iters))
                t_r.append(timer(ref_fn, args.iters))
                if args.plain:  # comparison kernel variant (tdl_gemm variant id)
                    gemm.VARIANT = args.plain_variant
                    t_p.append(timer(ours, args.iters))
                    gemm.VARIANT = 0
            tf = lambda t: round(fl / t / 1e12, 1)
            print(json.dumps({"shape": name, "prod": prod, "M": M, "K": K, "N": N, "relerr": round(err, 5),
                              "ours_tf_med": tf(statistics.median(t_o)), "ours_tf_best": tf(min(t_o)),
                              "torch_tf_med": tf(statistics.median(t_r)), "torch_tf_best": tf(min(t_r)),
                              "ratio": round(statistics.median(t_r) / statistics.median(t_o), 3),
                              **({"cmp_variant_tf_med": tf(statistics.median(t_p))} if t_p else {})}), flush=True)
            del ref


if __name__ == "__main__":
    main()
