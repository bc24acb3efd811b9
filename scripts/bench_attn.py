#!/usr/bin/env python3
"""Flash-attention microbenchmark (csrc/attention.hip): causal fwd / bwd TFLOP/s at GPT-2-medium
shapes (H=16, D=64, T=1024) on random data, vs torch SDPA (aten flash / math on ROCm)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops.layers import attn_bwd, attn_fwd  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    H, D, T = 16, 64, 1024
    for B, mode in ((8, ""), (8, "xcd"), (32, ""), (32, "xcd")):
        os.environ["TDL_ATTN_MAP"] = mode
        qkv = torch.randn(B, T, 3 * H * D, device="cuda").bfloat16()
        o, lse, scale = attn_fwd(qkv, H, True)
        do = torch.randn_like(o)
        fl = 4.0 * B * H * T * T * D / 2  # causal useful flops, fwd
        tf = timeit(lambda: attn_fwd(qkv, H, True))
        tb = timeit(lambda: attn_bwd(qkv, o, lse, do, H, True, scale))
        q, k, v = qkv.view(B, T, 3, H, D).permute(2, 0, 3, 1, 4)
        try:
            ts = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True))
        except Exception:  # noqa: BLE001
            ts = float("nan")
        print(json.dumps({"map": mode or "grid", "B": B, "H": H, "T": T, "D": D, "fwd_us": round(tf * 1e6, 1), "bwd_us": round(tb * 1e6, 1),
                          "fwd_tflops": round(fl / tf / 1e12, 1), "bwd_tflops": round(2.5 * fl / tb / 1e12, 1),
                          "torch_sdpa_fwd_tflops": round(fl / ts / 1e12, 1)}), flush=True)


if __name__ == "__main__":
    main()
