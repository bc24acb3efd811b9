#!/usr/bin/env python3
"""Interleaved in-process A/B of attention-forward variants selected per launch by an env var
(default TDL_ATTN_FWD_PF=1|2) at the bench shape (B=64, H=16, T=1024, D=64, causal): per-variant
us/call over rounds, TFLOP/s, and a bitwise check that the variants agree."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops.layers import attn_fwd  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    var = os.environ.get("AB_VAR", "TDL_ATTN_FWD_PF")
    vals = os.environ.get("AB_VALS", "1,2").split(",")
    B, H, D, T = int(os.environ.get("AB_B", "64")), 16, 64, 1024
    qkv = torch.randn(B, T, 3 * H * D, device="cuda").bfloat16()
    fl = 4.0 * B * H * T * T * D / 2
    outs = {}
    for v in vals:
        os.environ[var] = v
        outs[v] = attn_fwd(qkv, H, True)[0].clone()
    same = all(torch.equal(outs[vals[0]], outs[v]) for v in vals[1:])
    res = {v: [] for v in vals}
    for _ in range(5):
        for v in vals:
            os.environ[var] = v
            res[v].append(timeit(lambda: attn_fwd(qkv, H, True)))
    for v in vals:
        us = sorted(res[v])[len(res[v]) // 2]
        print(json.dumps({"var": var, "value": v, "B": B, "median_us": round(us, 1), "all_us": [round(x, 1) for x in res[v]],
                          "tflops": round(fl / us / 1e6, 1), "bitwise_equal_to_first": same}), flush=True)


if __name__ == "__main__":
    main()
