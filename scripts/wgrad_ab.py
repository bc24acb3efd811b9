#!/usr/bin/env python3
"""Weight-gradient kernel A/B at the N = 1 bench shape (64k tokens): for each GPT-2-medium product
fp32 main_grad += x^T dy, interleaved rounds of
  * the default (gemm_p4, TT operands read through ds_read_b64_tr_b16, split from the cost model),
  * tile-order variants (TDL_GEMM_GROUPM, read per launch),
  * the same product on pre-transposed operands (NT: x^T and dy^T stored k-contiguous) — the
    price of the transposed operand reads, not a routing option (the copies are not free).
One JSON line per (product, variant): median us over rounds, TF/s.

    python scripts/wgrad_ab.py --out gpurun_out/r6_wgrad_ab.jsonl
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import gemm  # noqa: E402

PRODUCTS = {"qkv": (1024, 3072), "o": (1024, 1024), "fc": (1024, 4096), "proj": (4096, 1024)}


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
    ap.add_argument("--K", type=int, default=65536)
    ap.add_argument("--products", default="qkv,o,fc,proj")
    ap.add_argument("--groups", default="0,2,4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--nt", type=int, default=1)
    ap.add_argument("--pd", type=int, default=0, help="also the LDS-DMA kernel (gemm_pd TT) at the default split")
    ap.add_argument("--out", default="gpurun_out/r6_wgrad_ab.jsonl")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    f = open(a.out, "a")
    K = a.K
    for name in a.products.split(","):
        M, N = PRODUCTS[name]
        torch.manual_seed(0)
        x = (torch.rand(K, M, device="cuda") * 2 - 1).bfloat16()
        dy = ((torch.rand(K, N, device="cuda") * 2 - 1) * 0.05).bfloat16()
        acc = torch.zeros(M, N, dtype=torch.float32, device="cuda")
        ref = x.float().t() @ dy.float()
        variants = {}
        for g in a.groups.split(","):
            def run(g=g):
                os.environ["TDL_GEMM_GROUPM"] = g
                gemm.matmul_f32_acc(acc, x.t(), dy)
            variants[f"tt_g{g}"] = run
        if a.pd:
            def run_pd():
                os.environ.pop("TDL_GEMM_GROUPM", None)
                gemm.matmul_f32_acc(acc, x.t(), dy, kernel="pd")
            variants["tt_pd"] = run_pd
        if a.nt:
            xt = x.t().contiguous()     # [M][K]
            dyt = dy.t().contiguous()   # [N][K]

            def run_nt():
                os.environ.pop("TDL_GEMM_GROUPM", None)
                gemm.matmul_f32_acc(acc, xt, dyt.t())
            variants["nt"] = run_nt
            if a.pd:
                def run_nt_pd():
                    os.environ.pop("TDL_GEMM_GROUPM", None)
                    gemm.matmul_f32_acc(acc, xt, dyt.t(), kernel="pd")
                variants["nt_pd"] = run_nt_pd
        # correctness of every variant once
        bad = {}
        for k, fn in variants.items():
            acc.zero_()
            fn()
            torch.cuda.synchronize()
            err = float((acc - ref).abs().max() / ref.abs().max())
            if err > 2e-2:
                bad[k] = err
        times = {k: [] for k in variants}
        for k, fn in variants.items():
            for _ in range(3):
                fn()
        for _ in range(a.rounds):
            for k, fn in variants.items():
                times[k].append(timed(fn, a.iters))
        os.environ.pop("TDL_GEMM_GROUPM", None)
        split = gemm.effective_split(K, gemm.wgrad_split(K, M, N))
        for k, ts in times.items():
            us = statistics.median(ts)
            rec = {"product": name, "M": M, "N": N, "K": K, "split": split, "variant": k, "us": round(us, 1),
                   "tflops": round(2.0 * M * N * K / us / 1e6, 1), "spread_us": round(max(ts) - min(ts), 1),
                   "bad": bad.get(k)}
            print(json.dumps(rec), flush=True)
            f.write(json.dumps(rec) + "\n")
        del x, dy, acc, ref
        torch.cuda.empty_cache()
    f.close()


if __name__ == "__main__":
    main()
