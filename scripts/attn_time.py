#!/usr/bin/env python3
"""Median us per call of the attention forward and backward at the bench shape (B=64 H=16
T=1024 D=64 causal) for whichever native library TDL_NATIVE_LIB selects (A/B across builds)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops.layers import attn_bwd, attn_fwd  # noqa: E402


def timeit(fn, iters=10, reps=5):
    for _ in range(3):
        fn()
    out = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / iters * 1e3)
    return sorted(out)[len(out) // 2]


B, H, T, D = int(os.environ.get("B", "64")), 16, 1024, 64
qkv = torch.randn(B, T, 3 * H * D, device="cuda").bfloat16()
o, lse, sc = attn_fwd(qkv, H, True)
do = torch.randn_like(o)
fl = 4.0 * B * H * T * T * D / 2
tf = timeit(lambda: attn_fwd(qkv, H, True))
tb = timeit(lambda: attn_bwd(qkv, o, lse, do, H, True, sc))
print(json.dumps({"lib": os.environ.get("TDL_NATIVE_LIB", "in-tree"), "fwd_us": round(tf, 1), "bwd_us": round(tb, 1),
                  "fwd_tflops": round(fl / tf / 1e6, 1), "bwd_tflops": round(2.5 * fl / tb / 1e6, 1)}), flush=True)
