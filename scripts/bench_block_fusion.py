#!/usr/bin/env python3
"""Fused GEMM epilogues vs library GEMM + separate elementwise pass, at the GPT-2 MLP shapes.

    fc forward:   torch.mm(h2, Wfc) -> tdl_bias_gelu_fwd          vs  gemm.matmul(epi='gelu')
    proj dgrad:   torch.mm(dy, Wp^T) -> tdl_bias_gelu_bwd (+ db)   vs  gemm.matmul(epi='dgelu', colsum)

Both paths are timed in interleaved rounds in one process on uniform random data; one JSON line
per product with the median ms of each path and the ratio (library path / fused path).

    python scripts/bench_block_fusion.py [--tokens 32768] [--model medium]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import _lib, gemm  # noqa: E402
from trustworthy_dl.ops import block  # noqa: E402


def timer(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--model", default="medium")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variant", type=int, default=0, help="tdl_gemm variant for the fused products (36 = LDS epilogue)")
    ap.add_argument("--nt", action="store_true", help="forward weight as the block stores it ([out, in] copy: NT)")
    args = ap.parse_args()
    gemm.VARIANT = args.variant
    _lib.lib()
    dev = torch.device("cuda:0")
    C = 1024 if args.model == "medium" else 768
    M = args.tokens
    r = lambda *s, sc=1.0: ((torch.rand(*s, device=dev) * 2 - 1) * sc).bfloat16()
    h2, wfc, bfc = r(M, C), r(C, 4 * C, sc=0.05), r(4 * C, sc=0.1)
    if args.nt:
        wfc = wfc.t().contiguous().t()
    dy, wp = r(M, C), r(4 * C, C, sc=0.05)
    pre_lib = torch.mm(h2, wfc)
    pre_fused = torch.empty_like(pre_lib)
    db = torch.zeros(4 * C, device=dev)

    def fc_lib():
        return block._bias_gelu_fwd(torch.mm(h2, wfc), bfc)

    def fc_fused():
        return gemm.matmul(h2, wfc, bias=bfc, epi="gelu", aux=pre_fused)

    def dg_lib():
        return block._bias_gelu_bwd(torch.mm(dy, wp.t()), pre_lib, bfc, db)

    def dg_fused():
        return gemm.matmul(dy, wp.t(), epi="dgelu", aux=pre_fused, colsum=db)

    from trustworthy_dl.ops import blaslt
    pre_bl = torch.empty_like(pre_lib)
    db_bl = torch.zeros(4 * C, device=dev)

    def fc_blaslt():
        y = torch.empty_like(pre_lib)
        assert blaslt.gemm_colmajor(0, 0, 4 * C, M, C, 1.0, wfc, 4 * C, h2, C, 0.0, y, 4 * C, y, 4 * C,
                                    blaslt.EPI_GELU_AUX_BIAS, bfc, pre_bl, 4 * C), "GELU_AUX_BIAS unsupported"
        return y

    def dg_blaslt():
        d = torch.empty_like(pre_lib)
        # dpre[M, 4C] = (dy[M, C] @ Wp^T) * gelu'(pre), bias grad of the result into db_bl
        assert blaslt.gemm_colmajor(1, 0, 4 * C, M, C, 1.0, wp, C, dy, C, 0.0, d, 4 * C, d, 4 * C,
                                    208, db_bl, pre_bl, 4 * C), "DGELU_BGRAD unsupported"
        return d

    # numerics: both paths against each other (fp32 reference checks live in tests/test_gemm_gpu.py)
    f1, f2 = fc_lib(), fc_fused()
    err_fc = float((f1.float() - f2.float()).abs().max() / f1.float().abs().max())
    d1, d2 = dg_lib(), dg_fused()
    err_dg = float((d1.float() - d2.float()).abs().max() / d1.float().abs().max())
    f3 = d3 = None
    try:
        f3 = fc_blaslt()
        err_fc_bl = float((f1.float() - f3.float()).abs().max() / f1.float().abs().max())
    except AssertionError as e:
        print(json.dumps({"note": str(e)}), flush=True)
    try:
        d3 = dg_blaslt()
        err_dg_bl = float((d1.float() - d3.float()).abs().max() / d1.float().abs().max())
    except AssertionError as e:
        print(json.dumps({"note": str(e)}), flush=True)
        err_dg_bl = None
    cases = [("fc_fwd_gelu", fc_lib, fc_fused, err_fc, 2.0 * M * C * 4 * C),
             ("proj_dgrad_dgelu", dg_lib, dg_fused, err_dg, 2.0 * M * C * 4 * C)]
    if f3 is not None:
        cases.append(("fc_fwd_gelu_blaslt_epilogue", fc_lib, fc_blaslt, err_fc_bl, 2.0 * M * C * 4 * C))
    if d3 is not None:
        cases.append(("proj_dgrad_dgelu_blaslt_epilogue", dg_lib, dg_blaslt, err_dg_bl, 2.0 * M * C * 4 * C))
    for name, lib_fn, fused_fn, err, fl in cases:
        t_l, t_f = [], []
        lib_fn(); fused_fn()
        for _ in range(args.rounds):
            t_l.append(timer(lib_fn, args.iters))
            t_f.append(timer(fused_fn, args.iters))
        ml, mf = statistics.median(t_l), statistics.median(t_f)
        print(json.dumps({"product": name, "M": M, "C": C, "lib_ms": round(ml, 4), "fused_ms": round(mf, 4),
                          "lib_tf": round(fl / ml / 1e9, 1), "fused_tf": round(fl / mf / 1e9, 1),
                          "speedup": round(ml / mf, 3), "relerr_vs_lib": round(err, 4)}), flush=True)


if __name__ == "__main__":
    main()
