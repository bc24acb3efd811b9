#!/usr/bin/env python3
"""Interleaved timing of the native GEMM's schedule variants (tdl_gemm variant ids, NT bf16 only)
against hipBLASLt on GPT-2-medium NT shapes.  Variants 6 and 7 are timing-only ablations (no DMA
wait / no barrier: wrong results), the rest are checked against fp32 torch."""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import gemm  # noqa: E402

NAMES = {0: "default", 1: "plain", 2: "pipe", 3: "pipe+interleave", 4: "pipe+b_early", 5: "pipe+b_early+interleave",
         6: "ABL_no_vmwait", 7: "ABL_no_vmwait_no_barrier", 8: "pipe+setprio", 9: "pipe+interleave+setprio",
         10: "k8wave", 11: "persistent4", 12: "persistent8",
         13: "P8_ABL_noDMA", 14: "P8_ABL_noLDSread", 16: "P8_ABL_nowait", 17: "P8_ABL_noDMA_nowait",
         18: "P8_ABL_mfma_only", 19: "persistent8_norot"}


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
    ap.add_argument("--variants", default="0,11,12")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    M = 32768
    shapes = [("fc_fwd", 1024, 4096), ("proj_fwd", 4096, 1024), ("qkv_fwd", 1024, 3072)]
    vs = [int(v) for v in args.variants.split(",")]
    for name, K, N in shapes:
        a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        bt = ((torch.rand(N, K, device=dev) * 2 - 1) * 0.05).bfloat16()
        ref = a.float() @ bt.float().t()
        errs = {}
        for v in vs:
            gemm.VARIANT = v
            out = gemm.matmul(a, bt.t())
            errs[v] = float((out.float() - ref).abs().max() / ref.abs().max())
        del ref
        gemm.VARIANT = 0
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
        row = {"shape": name, "K": K, "N": N, "torch_tf": round(fl / statistics.median(times[-1]) / 1e12, 1)}
        for v in vs:
            row[NAMES[v]] = {"tf": round(fl / statistics.median(times[v]) / 1e12, 1), "err": round(errs[v], 4)}
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
