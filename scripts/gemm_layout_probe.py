#!/usr/bin/env python3
"""Forward / dgrad GEMM throughput for the GPT-2-medium block shapes with the weight stored
[in, out] (HF layout, current) vs [out, in], with and without the bias epilogue (torch hipBLASLt).
One JSON line per (tokens, shape)."""
import json
import os

import torch


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
    return s.elapsed_time(e) / iters * 1e-3


def main():
    dev = torch.device("cuda:0")
    tokens = [int(t) for t in os.environ.get("TOKENS", "16384,32768").split(",")]
    shapes = [("qkv", 1024, 3072), ("o", 1024, 1024), ("fc", 1024, 4096), ("proj", 4096, 1024)]
    for M in tokens:
        for name, K, N in shapes:
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(K, N, device=dev) * 0.02).to(torch.bfloat16)   # [in, out]
            wt = w.t().contiguous()                                          # [out, in]
            b = torch.randn(N, device=dev).to(torch.bfloat16)
            dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
            tf = lambda t: round(2.0 * M * K * N / t / 1e12, 1)
            r = {"M": M, "shape": name, "K": K, "N": N,
                 "fwd_w_in_out": tf(timeit(lambda: torch.mm(x, w))),
                 "fwd_w_out_in": tf(timeit(lambda: torch.mm(x, wt.t()))),
                 "fwd_bias_w_in_out": tf(timeit(lambda: torch.addmm(b, x, w))),
                 "fwd_bias_w_out_in": tf(timeit(lambda: torch.addmm(b, x, wt.t()))),
                 "dgrad_w_in_out": tf(timeit(lambda: torch.mm(dy, w.t()))),
                 "dgrad_w_out_in": tf(timeit(lambda: torch.mm(dy, wt))),
                 "wgrad_in_out": tf(timeit(lambda: torch.mm(x.t(), dy))),
                 "wgrad_out_in": tf(timeit(lambda: torch.mm(dy.t(), x)))}
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
