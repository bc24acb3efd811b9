#!/usr/bin/env python3
"""Weight-gradient products of GPT-2-medium at 32k tokens (dW[in, out] += x^T dy into fp32):
the ping-pong native GEMM on transposed operands (tdl_gemm variant 20, TA = TB = 1) with split-K
slabs or fp32 atomics, vs the shipped library path (ops.layers.wgrad_acc: hipBLASLt batched GEMM
into fp32 slabs + native reduce) and the 8-wave native kernel.  Interleaved rounds in one process;
uniform random operands; every method checked against fp32 torch first."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import gemm, layers  # noqa: E402


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
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    T = args.tokens
    for name, cin, cout in [("qkv", 1024, 3072), ("o", 1024, 1024), ("fc", 1024, 4096), ("proj", 4096, 1024)]:
        torch.manual_seed(0)
        x = (torch.rand(T, cin, device=dev) * 2 - 1).bfloat16()
        dy = ((torch.rand(T, cout, device=dev) * 2 - 1) * 0.1).bfloat16()
        ref = x.float().t() @ dy.float()
        acc = torch.zeros(cin, cout, device=dev)
        tiles = (cin // 256) * (cout // 256)

        def m_lib():
            layers.wgrad_acc(acc, x.t(), dy)

        def make_native(variant, split, mode):
            def f():
                gemm.VARIANT = variant
                gemm.matmul_f32_acc(acc, x.t(), dy, split=split, mode=mode)
                gemm.VARIANT = 0
            return f

        methods = {"lib": m_lib, "v0_default": make_native(0, None, None)}
        for S in (1, 2, 4, 8, 16):
            if tiles * S > 1024 or (T // 64) % S:
                continue
            methods[f"pp_slab{S}"] = make_native(20, S, "slab")
            if S > 1:
                methods[f"pp_atomic{S}"] = make_native(20, S, "atomic")
        errs = {}
        for k, f in methods.items():
            acc.zero_()
            f()
            torch.cuda.synchronize()
            errs[k] = float((acc - ref).abs().max() / ref.abs().max())
        times = {k: [] for k in methods}
        for _ in range(args.rounds):
            for k, f in methods.items():
                times[k].append(timer(f, args.iters))
        fl = 2.0 * T * cin * cout
        row = {"shape": name, "tokens": T, "in": cin, "out": cout, "tiles": tiles}
        for k in methods:
            row[k] = {"tf": round(fl / statistics.median(times[k]) / 1e12, 1), "err": float(f"{errs[k]:.2e}")}
        best = max((k for k in methods if k.startswith("pp")), key=lambda k: row[k]["tf"])
        row["best_pp"] = best
        row["best_pp_vs_lib"] = round(row[best]["tf"] / row["lib"]["tf"], 3)
        print(json.dumps(row), flush=True)
        del x, dy, ref, acc


if __name__ == "__main__":
    main()
