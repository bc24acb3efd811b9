#!/usr/bin/env python3
"""GEMM solution tuning probe for the GPT-2-medium shapes: times each GEMM the model issues with
the library heuristic's solution, then with torch's TunableOp (hipBLASLt + rocBLAS solutions
benchmarked per shape), and writes the tuned table to ``$TDL_TUNE_FILE``.

One JSON line per (M, shape, op) with TFLOP/s before / after."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def cases(M, dev):
    out = []
    for name, K, N in (("qkv", 1024, 3072), ("o", 1024, 1024), ("fc", 1024, 4096), ("proj", 4096, 1024),
                       ("lmhead", 1024, 50304)):
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(K, N, device=dev) * 0.02).bfloat16()
        dy = torch.randn(M, N, device=dev).bfloat16()
        fl = 2.0 * M * K * N
        if name == "lmhead":  # logits = h @ wte^T (wte stored [V, n]); dgrad dh = dlogits @ wte
            wt = w.t().contiguous()
            out.append((name, "fwd", fl, lambda x=x, wt=wt: torch.mm(x, wt.t())))
            out.append((name, "dgrad", fl, lambda dy=dy, wt=wt: torch.mm(dy, wt)))
            out.append((name, "wgrad", fl, lambda dy=dy, x=x: torch.mm(dy.t(), x)))
            continue
        out.append((name, "fwd", fl, lambda x=x, w=w: torch.mm(x, w)))
        out.append((name, "dgrad", fl, lambda dy=dy, w=w: torch.mm(dy, w.t())))
        out.append((name, "wgrad_mm", fl, lambda x=x, dy=dy: torch.mm(x.t(), dy)))
        for S in (4, 8):
            a3 = x.view(S, M // S, K).transpose(1, 2)
            b3 = dy.view(S, M // S, N)
            part = torch.empty(S, K, N, device=dev)
            out.append((name, f"wgrad_bmm_f32_s{S}", fl,
                        lambda a3=a3, b3=b3, part=part: torch.bmm(a3, b3, out_dtype=torch.float32, out=part)))
    return out


def main():
    dev = torch.device("cuda:0")
    Ms = [int(t) for t in os.environ.get("TOKENS", "16384,32768").split(",")]
    base = {}
    for M in Ms:
        for name, op, fl, fn in cases(M, dev):
            base[(M, name, op)] = fl / timeit(fn) / 1e12
    tune_file = os.environ.get("TDL_TUNE_FILE", "gpurun_out/tunableop_results.csv")
    os.makedirs(os.path.dirname(tune_file) or ".", exist_ok=True)
    torch.cuda.tunable.set_filename(tune_file)
    torch.cuda.tunable.set_max_tuning_duration(int(os.environ.get("TUNE_MS", "30")))
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    for M in Ms:
        for name, op, fl, fn in cases(M, dev):
            t = timeit(fn)
            print(json.dumps({"M": M, "shape": name, "op": op, "heuristic_tflops": round(base[(M, name, op)], 1),
                              "tuned_tflops": round(fl / t / 1e12, 1)}), flush=True)
    torch.cuda.tunable.write_file()
    print(json.dumps({"tuned_file": tune_file, "entries": len(torch.cuda.tunable.get_results())}))


if __name__ == "__main__":
    main()
