#!/usr/bin/env python3
"""qkv + o and fc + proj weight gradients at the bench shape (GPT-2-medium, 64k / 16k tokens): the two separate
launches (each its own split from the cost model, slabs reduced) vs ONE grouped launch
(gemm.matmul_f32_acc_grouped), interleaved rounds, median us.  One JSON line per (tokens, variant).

    python scripts/wgrad_grouped_ab.py --out gpurun_out/r6_wgrad_grouped_ab.jsonl
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
    ap.add_argument("--tokens", default="65536,16384")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default="gpurun_out/r6_wgrad_grouped_ab.jsonl")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    f = open(a.out, "a")
    C = 1024
    pairs = {"attn": ((C, 3 * C), (C, C)), "mlp": ((C, 4 * C), (4 * C, C))}
    for K, (pair, ((m1, n1), (m2, n2))) in ((int(t), pp) for t in a.tokens.split(",") for pp in pairs.items()):
        torch.manual_seed(0)
        h = (torch.rand(K, m1, device="cuda") * 2 - 1).bfloat16()
        o = (torch.rand(K, m2, device="cuda") * 2 - 1).bfloat16()
        dqkv = ((torch.rand(K, n1, device="cuda") * 2 - 1) * 0.05).bfloat16()
        dy = ((torch.rand(K, n2, device="cuda") * 2 - 1) * 0.05).bfloat16()
        g1 = torch.zeros(m1, n1, device="cuda")
        g2 = torch.zeros(m2, n2, device="cuda")

        def separate():
            gemm.matmul_f32_acc(g1, h.t(), dqkv)
            gemm.matmul_f32_acc(g2, o.t(), dy)

        def grouped():
            assert gemm.matmul_f32_acc_grouped(g1, h.t(), dqkv, g2, o.t(), dy)
        variants = {"separate": separate, "grouped": grouped}
        times = {k: [] for k in variants}
        for fn in variants.values():
            for _ in range(3):
                fn()
        for _ in range(a.rounds):
            for k, fn in variants.items():
                times[k].append(timed(fn, a.iters))
        flop = 2.0 * K * (m1 * n1 + m2 * n2)
        for k, ts in times.items():
            us = statistics.median(ts)
            rec = {"tokens": K, "pair": pair, "variant": k, "us": round(us, 1), "tflops": round(flop / us / 1e6, 1),
                   "spread_us": round(max(ts) - min(ts), 1),
                   "split_separate": [gemm.wgrad_split(K, m1, n1), gemm.wgrad_split(K, m2, n2)],
                   "split_grouped": gemm.grouped_split(K, m1, n1, m2, n2)}
            print(json.dumps(rec), flush=True)
            f.write(json.dumps(rec) + "\n")
        del h, o, dqkv, dy, g1, g2
        torch.cuda.empty_cache()
    f.close()


if __name__ == "__main__":
    main()
