#!/usr/bin/env python3
"""MLP c_fc GEMM + bias-GELU: separate native pointwise kernels vs hipBLASLt fused epilogues.

fwd: torch.mm + tdl_bias_gelu_fwd   vs  GELU_AUX_BIAS epilogue (writes pre-activation as AUX)
bwd: torch.mm (dF = dY Wp^T) + tdl_bias_gelu_bwd (dpre + bias grad)  vs  DGELU_BGRAD epilogue.
Prints microseconds and max errors vs an fp32 torch reference; one JSON line per M."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import _lib, blaslt  # noqa: E402
from trustworthy_dl.ops._lib import ptr, stream_ptr  # noqa: E402
from trustworthy_dl.ops.layers import _scratch  # noqa: E402

EPI_DGELU_BGRAD = 208


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
    dev = torch.device("cuda:0")
    n, nf = 1024, 4096
    for M in (16384, 32768):
        h = torch.randn(M, n, device=dev).bfloat16()
        wfc = (torch.randn(n, nf, device=dev) * 0.03).bfloat16()
        bfc = (torch.randn(nf, device=dev) * 0.1).bfloat16()
        wp = (torch.randn(nf, n, device=dev) * 0.03).bfloat16()
        dy = torch.randn(M, n, device=dev).bfloat16()
        s = stream_ptr(dev)
        # ---- forward
        pre_a = torch.empty(M, nf, device=dev, dtype=torch.bfloat16)
        f_a = torch.empty_like(pre_a)

        def fwd_sep():
            torch.mm(h, wfc, out=pre_a)
            _lib.call("tdl_bias_gelu_fwd", ptr(pre_a), ptr(bfc), ptr(f_a), M, nf, s)
        pre_b = torch.empty_like(pre_a)
        f_b = torch.empty_like(pre_a)

        def fwd_epi():
            return blaslt.gemm_colmajor(0, 0, nf, M, n, 1.0, wfc, nf, h, n, 0.0, f_b, nf, f_b, nf,
                                        blaslt.EPI_GELU_AUX_BIAS, bfc, pre_b, nf)
        ok_f = fwd_epi()
        t_fs = timeit(fwd_sep)
        t_fe = timeit(fwd_epi) if ok_f else None
        ref_pre = h.float() @ wfc.float() + bfc.float()
        ref_f = F.gelu(ref_pre, approximate="tanh")
        err_f = float((f_b.float() - ref_f).abs().max()) if ok_f else None
        err_fs = float((f_a.float() - ref_f).abs().max())
        # ---- backward through c_proj and the GELU
        df = torch.empty(M, nf, device=dev, dtype=torch.bfloat16)
        dpre_a = torch.empty_like(df)
        db_a = torch.zeros(nf, device=dev)
        scratch = _scratch(((M + 15) // 16) * nf, dev)

        def bwd_sep():
            torch.mm(dy, wp.t(), out=df)
            _lib.call("tdl_bias_gelu_bwd", ptr(df), ptr(pre_a), ptr(bfc), ptr(dpre_a), ptr(db_a), M, nf,
                      ptr(scratch), s)
        pre_raw = (h.float() @ wfc.float()).bfloat16()  # GELU_AUX_BIAS stores pre incl. bias
        dpre_b = torch.empty_like(df)
        db_b = torch.zeros(nf, device=dev)

        def bwd_epi():
            return blaslt.gemm_colmajor(1, 0, nf, M, n, 1.0, wp, n, dy, n, 0.0, dpre_b, nf, dpre_b, nf,
                                        EPI_DGELU_BGRAD, db_b, pre_b, nf)
        ok_b = bwd_epi()
        t_bs = timeit(bwd_sep)
        t_be = timeit(bwd_epi) if ok_b else None
        u = ref_pre.clone().requires_grad_(True)
        F.gelu(u, approximate="tanh").backward(dy.float() @ wp.float().t())
        err_b = float((dpre_b.float() - u.grad).abs().max() / u.grad.abs().max()) if ok_b else None
        err_bs = float((dpre_a.float() - u.grad).abs().max() / u.grad.abs().max())
        err_db = float((db_b - u.grad.sum(0)).abs().max() / u.grad.sum(0).abs().max()) if ok_b else None
        del pre_raw
        print(json.dumps({"M": M, "fwd_sep_us": round(t_fs, 1), "fwd_epi_us": t_fe and round(t_fe, 1),
                          "bwd_sep_us": round(t_bs, 1), "bwd_epi_us": t_be and round(t_be, 1),
                          "fwd_err_sep": err_fs, "fwd_err_epi": err_f, "bwd_rel_err_sep": err_bs,
                          "bwd_rel_err_epi": err_b, "dbias_rel_err_epi": err_db}), flush=True)


if __name__ == "__main__":
    main()
