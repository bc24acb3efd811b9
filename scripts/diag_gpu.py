#!/usr/bin/env python3
"""Isolated GPU diagnostics: one case per process (``python scripts/diag_gpu.py CASE``), so a
faulting kernel is pinpointed and nothing after it runs.  Prints max relative error vs fp32 torch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


def case(name):
    from trustworthy_dl.ops import blaslt
    from trustworthy_dl.ops import _lib
    _lib.lib()
    dev = "cuda"
    torch.manual_seed(0)
    M, K, N = 512, 256, 1024
    x = torch.randn(M, K, device=dev).bfloat16()
    W = (torch.randn(K, N, device=dev) * 0.05).bfloat16()
    b = (torch.randn(N, device=dev) * 0.1).bfloat16()
    dy = torch.randn(M, N, device=dev).bfloat16()
    if name == "fwd":
        Y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        ok = blaslt.gemm_colmajor(0, 0, N, M, K, 1.0, W, N, x, K, 0.0, Y, N, Y, N)
        torch.cuda.synchronize()
        print("ok" if ok else "unsupported", rel(Y, x.float() @ W.float()) if ok else "")
    elif name == "dgrad":
        dX = torch.empty(M, K, dtype=torch.bfloat16, device=dev)
        ok = blaslt.gemm_colmajor(1, 0, K, M, N, 1.0, W, N, dy, N, 0.0, dX, K, dX, K)
        torch.cuda.synchronize()
        print("ok" if ok else "unsupported", rel(dX, dy.float() @ W.float().t()) if ok else "")
    elif name == "wgrad_f32_beta1":
        dW = torch.ones(K, N, device=dev)
        ok = blaslt.gemm_colmajor(0, 1, N, K, M, 1.0, dy, N, x, K, 1.0, dW, N, dW, N)
        torch.cuda.synchronize()
        print("ok" if ok else "unsupported", rel(dW, 1 + x.float().t() @ dy.float()) if ok else "")
    elif name == "bias":
        Y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        ok = blaslt.gemm_colmajor(0, 0, N, M, K, 1.0, W, N, x, K, 0.0, Y, N, Y, N, blaslt.EPI_BIAS, b)
        torch.cuda.synchronize()
        print("ok" if ok else "unsupported", rel(Y, x.float() @ W.float() + b.float()) if ok else "")
    elif name == "bgrada":
        dW = torch.zeros(K, N, device=dev)
        db = torch.zeros(N, device=dev)
        ok = blaslt.gemm_colmajor(0, 1, N, K, M, 1.0, dy, N, x, K, 1.0, dW, N, dW, N, blaslt.EPI_BGRADA, db)
        torch.cuda.synchronize()
        print("ok" if ok else "unsupported", (rel(dW, x.float().t() @ dy.float()), rel(db, dy.float().sum(0))) if ok else "")
    elif name == "gelu_aux_bias":
        Y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        pre = torch.empty_like(Y)
        ok = blaslt.gemm_colmajor(0, 0, N, M, K, 1.0, W, N, x, K, 0.0, Y, N, Y, N, blaslt.EPI_GELU_AUX_BIAS, b, pre, N)
        torch.cuda.synchronize()
        r = x.float() @ W.float() + b.float()
        print("ok" if ok else "unsupported",
              (rel(pre, r), rel(Y, torch.nn.functional.gelu(r, approximate="tanh"))) if ok else "")
    elif name == "linear_t":
        from trustworthy_dl.ops.layers import linear_t
        Wt = (torch.randn(N, K, device=dev) * 0.05).bfloat16().requires_grad_(True)
        xx = x.clone().requires_grad_(True)
        y = linear_t(xx, Wt)
        y.backward(dy)
        torch.cuda.synchronize()
        print("ok", rel(y, x.float() @ Wt.float().t()), rel(xx.grad, dy.float() @ Wt.float()),
              rel(Wt.grad, dy.float().t() @ x.float()))
    elif name in ("attn_fwd", "attn_bwd"):
        from trustworthy_dl.ops import causal_attention
        B, T, H, D = 2, 256, 4, 64
        qkv = torch.randn(B, T, 3 * H * D, device=dev).bfloat16().requires_grad_(True)
        o = causal_attention(qkv, H, True)
        torch.cuda.synchronize()
        xq = qkv.detach().float().requires_grad_(True)
        q, k, v = xq.view(B, T, 3, H, D).permute(2, 0, 3, 1, 4)
        ref = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, T, H * D)
        msg = ["ok", rel(o, ref)]
        if name == "attn_bwd":
            g = torch.randn_like(o)
            o.backward(g)
            torch.cuda.synchronize()
            ref.backward(g.float())
            msg.append(rel(qkv.grad, xq.grad))
        print(*msg)
    else:
        raise SystemExit(f"unknown case {name}")


if __name__ == "__main__":
    case(sys.argv[1])
