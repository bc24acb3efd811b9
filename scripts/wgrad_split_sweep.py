#!/usr/bin/env python3
"""Weight-gradient split-K sweep on the persistent kernel (gemm_p4): fp32 main_grad += x^T dy for the
GPT-2-medium products at the token counts the engine runs them at — K = 65536 (bench N = 1: one
micro-batch of 64 x 1024), 16384 (MP = 8 bench: micro-batches of 16 x 1024), 4096 (local-mode
configs: micro-batches of 4 x 1024) — for every split S, the slab reduce included.  One JSON line
per (product, K, S): us per call, TF/s.  Picks the split ``ops.gemm.wgrad_split`` should make.

    python scripts/wgrad_split_sweep.py --out gpurun_out/r6_wgrad_split_sweep.jsonl
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import gemm  # noqa: E402

PRODUCTS = {"qkv": (1024, 3072), "o": (1024, 1024), "fc": (1024, 4096), "proj": (4096, 1024), "lmhead": (1024, 50304)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--Ks", default="4096,16384,65536")
    ap.add_argument("--splits", default="1,2,4,8,16")
    ap.add_argument("--products", default="qkv,o,fc,proj")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--kernel", default=None, help="p4 | pd (default: ops.gemm.WGRAD_KERNEL)")
    ap.add_argument("--out", default="gpurun_out/r6_wgrad_split_sweep.jsonl")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    f = open(a.out, "a")
    for K in [int(k) for k in a.Ks.split(",")]:
        for name in a.products.split(","):
            M, N = PRODUCTS[name]
            x = (torch.rand(K, M, device="cuda") * 2 - 1).bfloat16()
            dy = ((torch.rand(K, N, device="cuda") * 2 - 1) * 0.05).bfloat16()
            acc = torch.zeros(M, N, dtype=torch.float32, device="cuda")
            default = gemm.effective_split(K, gemm.wgrad_split(K, M, N))
            best = None
            for S in [int(s) for s in a.splits.split(",")]:
                if gemm.effective_split(K, S) != S:
                    continue
                for _ in range(3):
                    gemm.matmul_f32_acc(acc, x.t(), dy, split=S, kernel=a.kernel)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.iters):
                    gemm.matmul_f32_acc(acc, x.t(), dy, split=S, kernel=a.kernel)
                e.record()
                e.synchronize()
                us = s.elapsed_time(e) * 1e3 / a.iters
                rec = {"product": name, "kernel": a.kernel or gemm.WGRAD_KERNEL, "M": M, "N": N, "K": K, "split": S,
                       "us": round(us, 1),
                       "tflops": round(2.0 * M * N * K / us / 1e6, 1), "default_split": default}
                best = rec if best is None or us < best["us"] else best
                print(json.dumps(rec), flush=True)
                f.write(json.dumps(rec) + "\n")
            print(json.dumps({"product": name, "K": K, "best_split": best["split"], "best_us": best["us"],
                              "default_split": default}), flush=True)
            del x, dy, acc
            torch.cuda.empty_cache()
    f.close()


if __name__ == "__main__":
    main()
