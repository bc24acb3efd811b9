#!/usr/bin/env python3
"""GEMM microbenchmark for the GPT-2-medium block shapes: forward / dgrad / weight-gradient variants
(torch hipBLASLt).  Weight-gradient variants: (a) addmm.dtype_out fp32 accumulate in place,
(b) bf16 mm + native fp32 add, (c) the transposed product dY^T.X (bf16) + transposed add.
One JSON line per shape with TFLOP/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import _lib  # noqa: E402
from trustworthy_dl.ops._lib import ptr, stream_ptr  # noqa: E402


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
    dev = torch.device("cuda:0")
    tokens = [int(t) for t in os.environ.get("TOKENS", "8192,32768").split(",")]
    shapes = [("qkv", 1024, 3072), ("o", 1024, 1024), ("fc", 1024, 4096), ("proj", 4096, 1024)]
    for M in tokens:
        for name, K, N in shapes:
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(K, N, device=dev) * 0.02).to(torch.bfloat16)
            dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
            acc = torch.zeros(K, N, device=dev)
            fl = 2.0 * M * K * N
            t_fwd = timeit(lambda: torch.mm(x, w))
            t_dgr = timeit(lambda: torch.mm(dy, w.t()))
            t_a = timeit(lambda: torch.ops.aten.addmm.dtype_out(acc, x.t(), dy, torch.float32, beta=1, alpha=1, out=acc))

            def var_b():
                g = torch.mm(x.t(), dy)
                _lib.call("tdl_add_into_f32", ptr(acc), ptr(g), g.numel(), 1, stream_ptr(dev))
            t_b = timeit(var_b)
            t_b_mm = timeit(lambda: torch.mm(x.t(), dy))
            t_c_mm = timeit(lambda: torch.mm(dy.t(), x))
            split = {}
            for S in (2, 4, 8):
                if M % S:
                    continue
                a3 = x.view(S, M // S, K).transpose(1, 2)
                b3 = dy.view(S, M // S, N)
                part = torch.empty(S, K, N, device=dev)

                def var_d():
                    try:
                        torch.bmm(a3, b3, out_dtype=torch.float32, out=part)
                    except TypeError:
                        torch.bmm(a3, b3, out=part.to(torch.bfloat16))
                    acc.add_(part.sum(0))
                split[S] = timeit(var_d)
            tf = lambda t: round(fl / t / 1e12, 1)
            print(json.dumps({"M": M, "shape": name, "K": K, "N": N, "fwd": tf(t_fwd), "dgrad": tf(t_dgr),
                              "wgrad_addmm_f32": tf(t_a), "wgrad_bf16_plus_add": tf(t_b),
                              "wgrad_bf16_mm_only": tf(t_b_mm), "wgrad_T_mm_only": tf(t_c_mm),
                              "wgrad_splitk_bmm_f32": {S: tf(t) for S, t in split.items()}}), flush=True)


if __name__ == "__main__":
    main()
