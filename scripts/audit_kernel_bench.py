#!/usr/bin/env python3
"""Throughput of the audit primitives on one GPU at the shapes of one GPT-2-medium MP = 8 stage
(~44 M fp32 gradient words, M = 16 micro-batch contributions): batched Merkle roots of the ring,
a single root, the keyed sketch of the ring, the contribution snapshot.  One JSON line per op.

    python scripts/audit_kernel_bench.py --out gpurun_out/audit_kernel_bench.jsonl
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.security import grad_audit as ga  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=44_000_000)
    ap.add_argument("--m", type=int, default=16)
    ap.add_argument("--out", default="gpurun_out/audit_kernel_bench.jsonl")
    a = ap.parse_args()
    n, M = a.n, a.m
    ring = torch.randn(M, n, device="cuda")
    g = torch.randn(n, device="cuda")
    prev = torch.randn(n, device="cuda")
    out = torch.empty(M, 8, dtype=torch.int32, device="cuda")
    recs = []

    def rec(op, ms, nbytes):
        r = {"op": op, "ms": round(ms, 4), "GB": round(nbytes / 1e9, 3), "TB_per_s": round(nbytes / ms / 1e9, 3)}
        print(json.dumps(r), flush=True)
        recs.append(r)
    rec("merkle_ring_batched", timeit(lambda: ga.merkle_roots(ring, [(0, n)], batch=M, stride=n, out=out)), 4 * M * n)
    rec("merkle_single", timeit(lambda: ga.merkle_roots(g, [(0, n)], out=out[:1])), 4 * n)
    rec("keyed_sketch_ring", timeit(lambda: ga.keyed_sketch(ring, [(0, n)], 12345, batch=M, stride=n)), 4 * M * n)
    rec("contrib_snap", timeit(lambda: ga.contrib_snap(g, prev, ring[0])), 16 * n)
    rec("copy", timeit(lambda: ring[1].copy_(g)), 8 * n)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        for r in recs:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
