#!/usr/bin/env python3
"""How much of gemm_pd's gap to the library on the K = 1024 forward products is its epilogue:
interleaved rounds of the library GEMM (torch.mm), gemm_pd (16-byte-store epilogue) and gemm_pd
with the epilogue compiled out (TDL_PD_SCHED=10, diagnostics: the output is not written).
One JSON line per (product, variant): median us, TF/s.

    python scripts/pd_epilogue_ab.py --out gpurun_out/r6_pd_epilogue_ab.jsonl
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import gemm  # noqa: E402

C = 1024
PRODUCTS = {"qkv_fwd": (C, 3 * C), "o_fwd": (C, C), "fc_fwd": (C, 4 * C), "proj_fwd": (4 * C, C),
            "lm_fwd": (C, 50304)}


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
    ap.add_argument("--tokens", type=int, default=65536)
    ap.add_argument("--only", default="qkv_fwd,o_fwd,fc_fwd,proj_fwd,lm_fwd")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--staggers", default="", help="extra gemm_pd variants: TDL_PD_STAGGER values, ';'-separated")
    ap.add_argument("--noepi", type=int, default=1)
    ap.add_argument("--kernels", default="", help="extra native kernels to time (p4, p4l, pp), comma-separated")
    ap.add_argument("--envs", default="", help="extra gemm_pd variants 'name:VAR=V,VAR2=V;...' (env per launch)")
    ap.add_argument("--out", default="gpurun_out/r6_pd_epilogue_ab.jsonl")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    f = open(a.out, "a")
    M = a.tokens
    gemm.KERNEL = "pd"
    for name in a.only.split(","):
        K, N = PRODUCTS[name]
        torch.manual_seed(0)
        x = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16()
        w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16()   # [out][in]: NT
        y = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
        iters = 3 if name == "lm_fwd" else 10

        def pd(v, st=""):
            def run():
                if v:
                    os.environ["TDL_PD_SCHED"] = v
                if st:
                    os.environ["TDL_PD_STAGGER"] = st
                gemm.matmul(x, w.t(), out=y)
                os.environ.pop("TDL_PD_SCHED", None)
                os.environ.pop("TDL_PD_STAGGER", None)
            return run
        variants = {"lib": lambda: torch.mm(x, w.t(), out=y), "pd": pd("")}
        if a.noepi:
            variants["pd_noepi"] = pd("10")
        for kn in [t for t in a.kernels.split(",") if t]:
            def run_kn(kn=kn):
                gemm.matmul(x, w.t(), out=y, kernel=kn)
            variants[kn] = run_kn
        for st in [t for t in a.staggers.split(";") if t]:
            variants[f"pd_st{st}"] = pd("", st)
        for spec in [t for t in a.envs.split(";") if t]:
            vname, kvs = spec.split(":", 1)
            env = dict(kv.split("=", 1) for kv in kvs.split(","))

            def run_env(env=env):
                old = {k: os.environ.get(k) for k in env}
                os.environ.update(env)
                gemm.matmul(x, w.t(), out=y)
                for k, v in old.items():
                    if v is None:
                        os.environ.pop(k, None)
                    else:
                        os.environ[k] = v
            variants[vname] = run_env
        times = {k: [] for k in variants}
        torch.mm(x, w.t(), out=y)
        ref = y.float().clone()
        errs = {}
        for k, fn in variants.items():
            y.zero_()
            fn()
            torch.cuda.synchronize()
            errs[k] = float((y.float() - ref).abs().max() / ref.abs().max())
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for k, fn in variants.items():
                times[k].append(timed(fn, iters))
        for k, ts in times.items():
            us = statistics.median(ts)
            rec = {"product": name, "M": M, "K": K, "N": N, "variant": k, "us": round(us, 1),
                   "tflops": round(2.0 * M * N * K / us / 1e6, 1), "spread_us": round(max(ts) - min(ts), 1),
                   "relerr_vs_lib": errs[k]}
            print(json.dumps(rec), flush=True)
            f.write(json.dumps(rec) + "\n")
        del x, w, y
        torch.cuda.empty_cache()
    f.close()


if __name__ == "__main__":
    main()
