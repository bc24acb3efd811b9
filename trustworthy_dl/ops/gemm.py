"""Native bf16 MFMA GEMM (csrc/gemm.hip) with fused epilogues.

``matmul(a, b)`` computes ``a @ b`` for a logical ``a [M, K]`` and ``b [K, N]`` whose storage may be
either row-major or a transposed view of a row-major tensor (the kernel reads both forms: k-contiguous
operands with ``ds_read_b128``, row-contiguous ones with the gfx950 transposing LDS read).  So every
product of a linear layer runs on the parameters as they are stored, with no transposed copies:

    forward   y  = x @ W             a = x,     b = W            (W [in, out], HF Conv1D)
    dgrad     dx = dy @ W.t()        a = dy,    b = W.t()
    wgrad     dW += x.t() @ dy       a = x.t(), b = dy           (fp32, into main_grad)

Epilogues (fused into the GEMM's store): ``bias``; ``gelu`` (stores the pre-activation too);
``resadd`` (out += a @ b, the residual stream); ``dgelu`` (out = (a @ b) * gelu'(pre), bias
gradient accumulated as fp32 column sums); fp32 ``acc`` / ``store`` / split-K ``atomic``.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from . import _lib
from ._lib import ptr, stream_ptr

EPI = {"none": 0, "gelu": 1, "resadd": 2, "dgelu": 3, "f32": 4, "f32acc": 5, "f32atomic": 6}
BK = 64
# Kernel (csrc/gemm.hip): "p4" = the persistent 4-wave kernel (one wave per SIMD owning 128 x 128,
# register-staged operands), "pp" = the staggered 8-wave ping-pong kernel (LDS-DMA staging,
# LDS-staged row-contiguous epilogue on NT operands), "pd" = the persistent 4-wave kernel with
# LDS-DMA staging on the library kernel's schedule (NT operands only).
KERNELS = {"p4": 0, "pp": 1, "p4l": 2, "pd": 3}
KERNEL = os.environ.get("TDL_GEMM_KERNEL", "pp")        # bf16-output products (matmul)
# the bias + GELU product (the MLP fc forward) on the LDS-DMA kernel's 16-byte-store epilogue: +0.4 %
# per step over the ping-pong kernel, 3 of 3 interleaved rounds (profiles/r5_gemm_pd_gelu_ab.txt)
GELU_KERNEL = os.environ.get("TDL_GEMM_GELU_KERNEL", "pd")
DGELU_KERNEL = os.environ.get("TDL_GEMM_DGELU_KERNEL", "")   # the dGELU product (proj dgrad); "" = KERNEL
# fp32 weight-gradient products (both operands row-contiguous: transposed LDS reads) on the LDS-DMA
# kernel: 7-10 % faster than the register-staged gemm_p4 on every GPT-2-medium weight gradient at
# 64k tokens once its copies stopped being drained in front of the transposed reads
# (profiles/r6_wgrad_pd_ab.jsonl)
WGRAD_KERNEL = os.environ.get("TDL_WGRAD_KERNEL", "pd")


def _operand_a(a: torch.Tensor):
    """(transposed_storage, ld) for a logical [M, K] operand."""
    if a.stride(1) == 1 and a.stride(0) >= a.shape[1]:
        return 0, a.stride(0)
    if a.stride(0) == 1 and a.stride(1) >= a.shape[0]:
        return 1, a.stride(1)
    raise ValueError(f"operand A needs a row-major or transposed-row-major layout (strides {a.stride()})")


def _operand_b(b: torch.Tensor):
    """(transposed_storage, ld) for a logical [K, N] operand: tb = 1 when stored [K][N]."""
    if b.stride(1) == 1 and b.stride(0) >= b.shape[1]:
        return 1, b.stride(0)
    if b.stride(0) == 1 and b.stride(1) >= b.shape[0]:
        return 0, b.stride(1)
    raise ValueError(f"operand B needs a row-major or transposed-row-major layout (strides {b.stride()})")


def supported(a: torch.Tensor, b: torch.Tensor) -> bool:
    """Shapes/layouts the native kernel takes (everything else stays on the caller's path)."""
    if not (a.is_cuda and a.dtype == torch.bfloat16 and b.dtype == torch.bfloat16 and a.dim() == 2 and b.dim() == 2):
        return False
    M, K = a.shape
    N = b.shape[1]
    if K % BK or K < 2 * BK or N % 8 or M % 8 or b.shape[0] != K:
        return False
    try:
        ta, lda = _operand_a(a)
        tb, ldb = _operand_b(b)
    except ValueError:
        return False
    return lda % 8 == 0 and ldb % 8 == 0 and a.data_ptr() % 16 == 0 and b.data_ptr() % 16 == 0


def _launch(a, b, c, ldc, epi, bias=None, aux=None, colsum=None, split=1, split_stride=0, kernel=None):
    M, K = a.shape
    N = b.shape[1]
    ta, lda = _operand_a(a)
    tb, ldb = _operand_b(b)
    kn = kernel or KERNEL
    if kn == "pd" and (ta != tb or (ta and not epi.startswith("f32"))):   # pd: NT, or TT with fp32 out
        kn = "pp"
    kid = KERNELS[kn]
    _lib.call("tdl_gemm", ptr(a), ptr(b), ptr(c), ptr(bias), ptr(aux), ptr(colsum), M, N, K, lda, ldb, ldc,
              ta, tb, EPI[epi] | (kid << 8), int(split), int(split_stride), stream_ptr(a.device))


def matmul(a: torch.Tensor, b: torch.Tensor, bias: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
           epi: str = "none", aux: Optional[torch.Tensor] = None, colsum: Optional[torch.Tensor] = None,
           kernel: Optional[str] = None) -> torch.Tensor:
    """bf16 ``epi(a @ b)``.  ``epi='gelu'`` needs ``aux`` (receives the pre-activation, shape of the
    output); ``'resadd'`` adds into ``out``; ``'dgelu'`` reads the pre-activation from ``aux`` and
    accumulates the column sums of the result into ``colsum`` (fp32) when given.  ``kernel``
    overrides the per-epilogue choice (``KERNELS``)."""
    M, K = a.shape
    N = b.shape[1]
    if out is None:
        if epi == "resadd":
            raise ValueError("resadd needs out")
        out = torch.empty(M, N, dtype=torch.bfloat16, device=a.device)
    if out.stride(1) != 1:
        raise ValueError("out must be row-major")
    if epi in ("gelu", "dgelu") and (aux is None or aux.stride() != out.stride()):
        raise ValueError(f"{epi} needs aux with the output's layout")
    if epi == "dgelu" and _operand_a(a)[0]:
        raise ValueError("dgelu needs a row-major A (rows past M must read as zero for the column sums)")
    if kernel is None:
        kernel = (GELU_KERNEL or None) if epi == "gelu" else (DGELU_KERNEL or None) if epi == "dgelu" else None
    _launch(a, b, out, out.stride(0), epi, bias=bias, aux=aux, colsum=colsum, kernel=kernel)
    return out


def num_cus(device=None) -> int:
    try:
        return torch.cuda.get_device_properties(device or torch.cuda.current_device()).multi_processor_count
    except (RuntimeError, AssertionError):
        return 256


def wgrad_split(K: int, M: int, N: int, num_cu: Optional[int] = None) -> int:
    """Split of the reduction depth K of an fp32 product [M, K] @ [K, N] (a weight gradient: K =
    tokens) for the persistent kernel, from a cost model fitted to a sweep of every GPT-2-medium
    product at K = 4k / 16k / 64k tokens (profiles/r6_wgrad_split_sweep.jsonl, it picks the measured
    best split in all 12 cases):

        T(S) = rounds(S) x (K / S / 64 K steps x 1.5 us + 5 us) + [S > 1] S x M x N x 8 B / 5 TB/s

    (work items = tiles x S over the CUs in whole rounds; a split of S > 1 writes and re-reads S fp32
    slabs).  The occupancy-first rule it replaces took 16 slices for qkv at 16k tokens (the MP = 8
    micro-batch), 30 % slower than 4 there."""
    if os.environ.get("TDL_WGRAD_SPLITK", "1") == "0":
        return 1
    cu = num_cu or num_cus()
    tiles = ((M + 255) // 256) * ((N + 255) // 256)
    best, best_t = 1, float("inf")
    for s in (1, 2, 4, 8, 16):
        if s > 1 and effective_split(K, s) != s:
            continue
        rounds = -(-(tiles * s) // cu)
        t = rounds * ((K // s // BK) * 1.5 + 5.0) + (s * M * N * 8 / 5e6 if s > 1 else 0.0)
        if t < best_t - 1e-9:
            best, best_t = s, t
    return best


def matmul_f32_acc(acc: torch.Tensor, a: torch.Tensor, b: torch.Tensor, split: Optional[int] = None,
                   mode: Optional[str] = None, kernel: Optional[str] = None, sink=None) -> torch.Tensor:
    """``acc (fp32) += a @ b``.  With a split reduction the partial products go to fp32 slabs
    reduced by one native pass (``mode='slab'``, default) or straight into ``acc`` with fp32
    atomics (``mode='atomic'``).  ``sink(slabs, S) -> bool`` (the gradient verifier's fused
    reduce: this is the parameter's last accumulation of the step) may take over the slab reduce."""
    M, K = a.shape
    N = b.shape[1]
    if acc.dtype != torch.float32 or tuple(acc.shape) != (M, N) or not acc.is_contiguous():
        raise ValueError("acc must be a contiguous fp32 [M, N] buffer")
    kernel = kernel or WGRAD_KERNEL
    S = wgrad_split(K, M, N) if split is None else max(1, int(split))
    S = effective_split(K, S)
    mode = mode or os.environ.get("TDL_WGRAD_REDUCE", "slab")
    if S <= 1:
        _launch(a, b, acc, N, "f32acc", kernel=kernel)
        return acc
    if mode == "atomic":
        _launch(a, b, acc, N, "f32atomic", split=S, kernel=kernel)
        return acc
    slabs = torch.empty(S, M, N, dtype=torch.float32, device=acc.device)
    _launch(a, b, slabs, N, "f32", split=S, split_stride=M * N, kernel=kernel)
    if sink is not None and sink(slabs, S):
        return acc
    _lib.call("tdl_splitk_reduce_add", ptr(acc), ptr(slabs), S, acc.numel(), stream_ptr(acc.device))
    return acc


# two weight gradients with the same token count (the attention's qkv and o products; the MLP's fc
# and proj) in ONE launch of the LDS-DMA kernel, one output tile x slice per workgroup: the two
# launches' partial last rounds become one full round
WGRAD_GROUPED = os.environ.get("TDL_WGRAD_GROUPED", "1") != "0"


def grouped_split(K: int, M1: int, N1: int, M2: int, N2: int, num_cu: Optional[int] = None) -> int:
    """Split for the grouped pair (csrc/gemm.hip tdl_gemm_wgrad_grouped): the wgrad_split cost model
    over the pair's tiles, restricted to splits >= 2 whose work items fit ONE round on the CUs (the
    kernel runs one item per workgroup); 0 when none does."""
    cu = num_cu or num_cus()
    tiles = ((M1 + 255) // 256) * ((N1 + 255) // 256) + ((M2 + 255) // 256) * ((N2 + 255) // 256)
    best, best_t = 0, float("inf")
    for s in (2, 4, 8, 16):
        if effective_split(K, s) != s or tiles * s > cu:
            continue
        t = (K // s // BK) * 1.5 + 5.0 + s * (M1 * N1 + M2 * N2) * 8 / 5e6
        if t < best_t - 1e-9:
            best, best_t = s, t
    return best


def matmul_f32_acc_grouped(acc1: torch.Tensor, a1: torch.Tensor, b1: torch.Tensor, acc2: torch.Tensor,
                           a2: torch.Tensor, b2: torch.Tensor, sink1=None, sink2=None) -> bool:
    """``acc1 += a1 @ b1`` and ``acc2 += a2 @ b2`` (fp32, weight-gradient layout: both operands
    row-contiguous, same K) from one grouped launch, each product's slabs reduced by its own
    pass (or taken by its sink).  Returns False, having done nothing, when the pair does not qualify
    (the caller runs the two products separately)."""
    if not WGRAD_GROUPED or WGRAD_KERNEL != "pd":
        return False
    M1, K = a1.shape
    M2 = a2.shape[0]
    N1, N2 = b1.shape[1], b2.shape[1]
    if a2.shape[1] != K or b2.shape[0] != K or b1.shape[0] != K:
        return False
    for acc, m, n in ((acc1, M1, N1), (acc2, M2, N2)):
        if acc.dtype != torch.float32 or tuple(acc.shape) != (m, n) or not acc.is_contiguous():
            return False
    if not (supported(a1, b1) and supported(a2, b2)):
        return False
    (ta1, lda1), (tb1, ldb1) = _operand_a(a1), _operand_b(b1)
    (ta2, lda2), (tb2, ldb2) = _operand_a(a2), _operand_b(b2)
    if not (ta1 and tb1 and ta2 and tb2):
        return False
    S = grouped_split(K, M1, N1, M2, N2)
    if S < 2:
        return False
    slabs = torch.empty(S * (M1 * N1 + M2 * N2), dtype=torch.float32, device=acc1.device)
    s1 = slabs[:S * M1 * N1].view(S, M1, N1)
    s2 = slabs[S * M1 * N1:].view(S, M2, N2)
    st = stream_ptr(acc1.device)
    _lib.call("tdl_gemm_wgrad_grouped", ptr(a1), ptr(b1), ptr(s1), M1, N1, lda1, ldb1, ptr(a2), ptr(b2), ptr(s2),
              M2, N2, lda2, ldb2, K, S, st)
    for acc, sl, sink in ((acc1, s1, sink1), (acc2, s2, sink2)):
        if sink is not None and sink(sl, S):
            continue
        _lib.call("tdl_splitk_reduce_add", ptr(acc), ptr(sl), S, acc.numel(), st)
    return True


def effective_split(K: int, split: int) -> int:
    """The split the kernel runs: the largest value <= ``split`` dividing the K / 64 steps with at
    least two steps per slice (every slice the same depth; both kernels need a distinct first and
    last K step; mirrors tdl_gemm)."""
    steps = K // BK
    s = max(1, min(int(split), steps // 2))
    while s > 1 and steps % s:
        s -= 1
    return s
