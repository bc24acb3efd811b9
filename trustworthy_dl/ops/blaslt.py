"""Row-major linear layers on hipBLASLt (csrc/blaslt.hip).

Row-major ``Y[M,N] = X[M,K] @ W[K,N]`` is the column-major product ``Y^T = W^T X^T``, so every
call swaps the operands.  Weight-gradient GEMMs accumulate into the parameter's fp32
``main_grad`` with beta=1 (bf16 A/B, fp32 C/D).  A signature that hipBLASLt cannot serve
(no algorithm for an epilogue/type combination) is remembered and routed to an equivalent
unfused sequence — still GPU-native, never a silent CPU fallback.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional, Tuple

import torch

from . import _lib
from ._lib import ptr, stream_ptr

EPI_DEFAULT, EPI_BIAS, EPI_GELU_AUX_BIAS, EPI_BGRADA = 1, 4, 164, 256
_T = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}
_WS: Dict[int, torch.Tensor] = {}
_WS_BYTES = 64 << 20
_unsupported = set()
_declared = False


def _fn():
    global _declared
    l = _lib.lib()
    f = l.tdl_blaslt_gemm
    if not _declared:
        P, I, F, L = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_int64
        f.argtypes = [I, I, I, I, I, F, P, I, I, P, I, I, F, P, I, I, P, I, I, I, P, I, P, I, P, L, P]
        f.restype = ctypes.c_int
        _declared = True
    return f


def _ws(dev: torch.device) -> torch.Tensor:
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    w = _WS.get(idx)
    if w is None:
        w = torch.empty(_WS_BYTES, dtype=torch.uint8, device=dev)
        _WS[idx] = w
    return w


def gemm_colmajor(opA: int, opB: int, m: int, n: int, k: int, alpha: float, A, lda: int, B, ldb: int,
                  beta: float, C, ldc: int, D, ldd: int, epilogue: int = EPI_DEFAULT, bias=None,
                  aux=None, ld_aux: int = 0) -> bool:
    """Raw column-major hipBLASLt GEMM. Returns False if the configuration is unsupported."""
    sig = (opA, opB, m, n, k, lda, ldb, ldc, ldd, A.dtype, B.dtype, C.dtype, D.dtype, epilogue,
           None if bias is None else bias.dtype)
    if sig in _unsupported:
        return False
    ws = _ws(D.device)
    rc = _fn()(opA, opB, m, n, k, alpha, ptr(A), lda, _T[A.dtype], ptr(B), ldb, _T[B.dtype], beta,
               ptr(C), ldc, _T[C.dtype], ptr(D), ldd, _T[D.dtype], epilogue, ptr(bias),
               _T[bias.dtype] if bias is not None else 0, ptr(aux), ld_aux, ptr(ws), ws.numel(),
               stream_ptr(D.device))
    if rc == 2:
        _unsupported.add(sig)
        return False
    if rc != 0:
        raise RuntimeError(f"hipBLASLt gemm failed (code {rc}) for signature {sig}")
    return True


def mm(X: torch.Tensor, W: torch.Tensor, out: Optional[torch.Tensor] = None,
       bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Row-major Y = X @ W (+ bias)."""
    M, K = X.shape
    N = W.shape[1]
    Y = out if out is not None else torch.empty(M, N, dtype=X.dtype, device=X.device)
    ok = gemm_colmajor(0, 0, N, M, K, 1.0, W, N, X, K, 0.0, Y, N, Y, N,
                       EPI_BIAS if bias is not None else EPI_DEFAULT, bias)
    if not ok:
        if bias is not None:
            torch.addmm(bias, X, W, out=Y)
        else:
            torch.mm(X, W, out=Y)
    return Y


def linear_fwd(x2: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor], act: Optional[str]
               ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    M, K = x2.shape
    N = W.shape[1]
    if act == "gelu":
        y = torch.empty(M, N, dtype=x2.dtype, device=x2.device)
        pre = torch.empty_like(y)
        if bias is not None and gemm_colmajor(0, 0, N, M, K, 1.0, W, N, x2, K, 0.0, y, N, y, N,
                                              EPI_GELU_AUX_BIAS, bias, pre, N):
            return y, pre
        mm(x2, W, out=pre, bias=bias)
        _gelu_inplace_copy(pre, y)  # bias already folded into pre: GELU only
        return y, pre
    return mm(x2, W, bias=bias), None


_zero_bias: Dict[Tuple[int, int], torch.Tensor] = {}


def _zeros_bias(n: int, dev: torch.device) -> torch.Tensor:
    key = (n, dev.index or 0)
    z = _zero_bias.get(key)
    if z is None:
        z = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        _zero_bias[key] = z
    return z


def _gelu_inplace_copy(pre: torch.Tensor, y: torch.Tensor):
    M, N = pre.shape
    _lib.call("tdl_bias_gelu_fwd", ptr(pre), ptr(_zeros_bias(N, pre.device)), ptr(y), M, N, stream_ptr(pre.device))


def linear_bwd(x2: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor], pre: Optional[torch.Tensor],
               dy2: torch.Tensor, act: Optional[str], need_dx: bool):
    """Returns (dx, grad_W or None, grad_b or None); W/b grads go to main_grad when present."""
    M, K = x2.shape
    N = W.shape[1]
    dev = x2.device
    bias_done = False
    mg_b = getattr(bias, "main_grad", None) if bias is not None else None
    db_tmp = None
    if act == "gelu":
        dpre = torch.empty_like(pre)
        db_tmp = mg_b if mg_b is not None else (torch.zeros(N, dtype=torch.float32, device=dev)
                                                if bias is not None else None)
        from .layers import _scratch
        _lib.call("tdl_bias_gelu_bwd", ptr(dy2), ptr(pre), None, ptr(dpre), ptr(db_tmp), M, N,
                  ptr(_scratch(((M + 15) // 16) * N, dev)), stream_ptr(dev))
        dy2 = dpre
        bias_done = True

    dx = None
    if need_dx:
        dx = torch.empty(M, K, dtype=dy2.dtype, device=dev)
        if not gemm_colmajor(1, 0, K, M, N, 1.0, W, N, dy2, N, 0.0, dx, K, dx, K):
            torch.mm(dy2, W.t(), out=dx)

    # weight gradient: dW^T[N,K] (+)= dY^T[N,M] . X[M,K]
    mg_w = getattr(W, "main_grad", None)
    if mg_w is not None:
        dW, beta = mg_w, 1.0
    else:
        dW, beta = torch.zeros(K, N, dtype=torch.float32, device=dev), 0.0
    want_bgrad = bias is not None and not bias_done
    db_out = torch.empty(N, dtype=torch.float32, device=dev) if want_bgrad else None
    ok = gemm_colmajor(0, 1, N, K, M, 1.0, dy2, N, x2, K, beta, dW, N, dW, N,
                       EPI_BGRADA if want_bgrad else EPI_DEFAULT, db_out)
    if not ok and want_bgrad:
        ok = gemm_colmajor(0, 1, N, K, M, 1.0, dy2, N, x2, K, beta, dW, N, dW, N)
        if ok:
            db_out = dy2.float().sum(0)
    if not ok:
        dW.add_(torch.mm(x2.t(), dy2).float())
        if want_bgrad:
            db_out = dy2.float().sum(0)
    gw = None if mg_w is not None else dW.to(W.dtype)

    gb = None
    if bias is not None:
        if bias_done:
            gb = None if mg_b is not None else db_tmp.to(bias.dtype)
        elif mg_b is not None:
            mg_b.add_(db_out)
        else:
            gb = db_out.to(bias.dtype)
    return dx, gw, gb


def linear_t_fwd(x2: torch.Tensor, W: torch.Tensor) -> torch.Tensor:
    """Y[M,N] = X[M,K] @ W^T with W stored [N, K]."""
    M, K = x2.shape
    N = W.shape[0]
    Y = torch.empty(M, N, dtype=x2.dtype, device=x2.device)
    if not gemm_colmajor(1, 0, N, M, K, 1.0, W, K, x2, K, 0.0, Y, N, Y, N):
        torch.mm(x2, W.t(), out=Y)
    return Y


def linear_t_bwd(x2: torch.Tensor, W: torch.Tensor, dy2: torch.Tensor, need_dx: bool):
    M, K = x2.shape
    N = W.shape[0]
    dev = x2.device
    dx = None
    if need_dx:
        dx = torch.empty(M, K, dtype=dy2.dtype, device=dev)
        if not gemm_colmajor(0, 0, K, M, N, 1.0, W, K, dy2, N, 0.0, dx, K, dx, K):
            torch.mm(dy2, W, out=dx)
    mg = getattr(W, "main_grad", None)
    if mg is not None:
        dW, beta = mg, 1.0
    else:
        dW, beta = torch.zeros(N, K, dtype=torch.float32, device=dev), 0.0
    if not gemm_colmajor(0, 1, K, N, M, 1.0, x2, K, dy2, N, beta, dW, K, dW, K):
        dW.add_(torch.mm(dy2.t(), x2).float())
    return dx, (None if mg is not None else dW.to(W.dtype))
