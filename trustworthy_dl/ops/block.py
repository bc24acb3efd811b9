"""Fused pre-LN transformer block (GPT-2) as ONE autograd node with a hand-scheduled backward.

The reference builds its stages from HuggingFace ``GPT2Block`` modules (distributed_trainer.py:118-135)
and lets autograd run them op by op.  Here the whole block

    h1 = LN1(x);  qkv = h1 @ Wqkv + bqkv;  o = attn(qkv);  y1 = x + o @ Wo + bo
    h2 = LN2(y1); f = gelu(h2 @ Wfc + bfc);  y = y1 + f @ Wp + bp

is one ``torch.autograd.Function`` whose forward/backward call the gfx950 kernels directly, so that

* the residual adds disappear into neighbouring kernels: forward ``y1 = x + o@Wo + bo`` and
  ``LN2(y1)`` are one pass (``tdl_add_bias_ln_fwd``, which also pre-adds ``bp`` so the last GEMM
  accumulates onto the residual stream in place); backward ``dy1 = dy + LN2_bwd(dh2)`` and
  ``dx = dy1 + LN1_bwd(dh1)`` are computed inside the LayerNorm-backward kernel (``dres``);
* the bias gradients of the two residual-stream projections (``bp`` = colsum(dy), ``bo`` =
  colsum(dy1)) are column partials of that same LayerNorm-backward pass, not separate reductions;
* weight gradients accumulate in fp32 straight into ``param.main_grad`` (GEMM beta=1 epilogue);
* the MLP's elementwise work rides in the native MFMA GEMM's epilogue (csrc/gemm.hip, ping-pong
  kernel with LDS-staged row-contiguous epilogues): forward ``f = gelu(h2 @ Wfc + bfc)`` stores the
  pre-activation and the activation from one kernel, backward ``dpre = (dy @ Wp^T) * gelu'(pre)``
  accumulates the ``bfc`` gradient as column sums in the same kernel (1.005x / 1.20x of hipBLASLt +
  the separate pass, profiles/r2_gemm_fused_lds_epilogue.jsonl; +1.5 % per step,
  profiles/r2_native_mlp_ab.txt); every weight gradient runs on the native persistent kernel;
* autograd bookkeeping is one node per block instead of ~12 (host time matters at 8 stages x
  64 micro-batches per step).

CPU tensors run the same schedule with PyTorch reference primitives (what the CPU tests check
against the unfused module composition).
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import ptr, stream_ptr
from .layers import (_f32_acc, _scratch, _wants_main_grad, attn_bwd, attn_fwd, bump_weight_generation,  # noqa: F401
                     fwd_weight, run_or_defer, take_stats_sink, wgrad_acc, wgrad_acc_pair)

_FUSED_WIDTHS = (256, 512, 768, 1024, 1280, 1536, 2048)


def gemm_grouped_wgrad(branch: str) -> bool:
    """the branch's two weight gradients (attn: qkv + o, mlp: fc + proj) as one grouped launch
    (gemm.matmul_f32_acc_grouped); TDL_WGRAD_GROUPED_MLP=0 keeps the MLP pair separate"""
    from . import gemm
    if branch == "mlp" and os.environ.get("TDL_WGRAD_GROUPED_MLP", "1") == "0":
        return False
    return gemm.WGRAD_GROUPED and gemm.WGRAD_KERNEL == "pd"


def fused_block_enabled(width: int, device: torch.device) -> bool:
    if os.environ.get("TDL_FUSED_BLOCK", "1") == "0":
        return False
    return device.type == "cpu" or width in _FUSED_WIDTHS


# ---------------------------------------------------------------- primitives (GPU kernel | CPU reference)
def _ln_fwd(x2, w, b, eps):
    M, N = x2.shape
    if x2.is_cuda:
        y = torch.empty_like(x2)
        mean = torch.empty(M, dtype=torch.float32, device=x2.device)
        rstd = torch.empty_like(mean)
        _lib.call("tdl_layernorm_fwd", ptr(x2), ptr(w), ptr(b), ptr(y), ptr(mean), ptr(rstd), M, N, float(eps),
                  stream_ptr(x2.device))
        return y, mean, rstd
    xf = x2.float()
    mean = xf.mean(-1)
    rstd = torch.rsqrt(xf.var(-1, unbiased=False) + eps)
    return ((xf - mean[:, None]) * rstd[:, None] * w.float() + b.float()).to(x2.dtype), mean, rstd


def _add_bias_ln_fwd(x2, z, bz, b2, w, b, eps, y1b_shape=None):
    """(y1 = x + z + bz, y1b = y1 + b2, h = LN(y1), mean, rstd); y1b is allocated with
    ``y1b_shape`` (a base tensor, not a view: it becomes the block's output)."""
    M, N = x2.shape
    y1b = torch.empty(y1b_shape or (M, N), dtype=x2.dtype, device=x2.device)
    if x2.is_cuda:
        y1 = torch.empty_like(x2)
        h = torch.empty_like(x2)
        mean = torch.empty(M, dtype=torch.float32, device=x2.device)
        rstd = torch.empty_like(mean)
        _lib.call("tdl_add_bias_ln_fwd", ptr(x2), ptr(z), ptr(bz), ptr(b2), ptr(w), ptr(b), ptr(y1), ptr(y1b),
                  ptr(h), ptr(mean), ptr(rstd), M, N, float(eps), stream_ptr(x2.device))
        return y1, y1b, h, mean, rstd
    y1 = (x2.float() + z.float() + bz.float()).to(x2.dtype)
    y1b.view(M, N).copy_(y1.float() + b2.float())
    h, mean, rstd = _ln_fwd(y1, w, b, eps)
    return y1, y1b, h, mean, rstd


def _ln_bwd(dy, x2, w, mean, rstd, dw_acc, db_acc, dres=None, sres_acc=None, sdx_acc=None):
    """dx = LN_bwd(dy) + dres; dgamma/dbeta and (optionally) colsum(dres), colsum(dx) accumulated."""
    M, N = x2.shape
    if dy.is_cuda:
        dx = torch.empty_like(x2)
        ws = int(_lib.lib().tdl_layernorm_bwd_ws_floats(M, N))
        _lib.call("tdl_layernorm_bwd_res", ptr(dy), ptr(x2), ptr(w), ptr(mean), ptr(rstd), ptr(dres), ptr(dx),
                  ptr(dw_acc), ptr(db_acc), ptr(sres_acc), ptr(sdx_acc), M, N, ptr(_scratch(ws, dy.device)),
                  stream_ptr(dy.device))
        return dx
    xf, g = x2.float(), dy.float()
    xh = (xf - mean[:, None]) * rstd[:, None]
    gw = g * w.float()
    dxf = rstd[:, None] * (gw - gw.mean(-1, keepdim=True) - xh * (gw * xh).mean(-1, keepdim=True))
    dw_acc.add_((g * xh).sum(0))
    db_acc.add_(g.sum(0))
    if dres is not None:
        dxf = dxf + dres.float()
    dx = dxf.to(dy.dtype)
    if sres_acc is not None:
        sres_acc.add_(dres.float().sum(0))
    if sdx_acc is not None:
        sdx_acc.add_(dx.float().sum(0))
    return dx


def _bias_gelu_fwd(pre, b):
    if pre.is_cuda:
        f = torch.empty_like(pre)
        _lib.call("tdl_bias_gelu_fwd", ptr(pre), ptr(b), ptr(f), pre.shape[0], pre.shape[1], stream_ptr(pre.device))
        return f
    return F.gelu(pre.float() + b.float(), approximate="tanh").to(pre.dtype)


def _bias_gelu_bwd(df, pre, b, db_acc):
    M, N = pre.shape
    if pre.is_cuda:
        dpre = torch.empty_like(pre)
        _lib.call("tdl_bias_gelu_bwd", ptr(df), ptr(pre), ptr(b), ptr(dpre), ptr(db_acc), M, N,
                  ptr(_scratch(((M + 15) // 16) * N, pre.device)), stream_ptr(pre.device))
        return dpre
    u = (pre.float() + b.float()).requires_grad_(True)
    with torch.enable_grad():
        out = F.gelu(u, approximate="tanh")
    (g,) = torch.autograd.grad(out, u, df.float())
    db_acc.add_(g.sum(0))
    return g.to(pre.dtype)


def _colsum_into(acc, d):
    M, N = d.shape
    if d.is_cuda and d.dtype == torch.bfloat16 and N % 8 == 0:
        _lib.call("tdl_colsum_bf16", ptr(d), ptr(acc), M, N, ptr(_scratch(((M + 15) // 16) * N, d.device)),
                  stream_ptr(d.device))
    else:
        acc.add_(d.float().sum(0))


# GEMM routing (fixed, measured): products with an elementwise epilogue to fuse (the MLP's fc forward
# with bias + GELU, its proj dgrad with dGELU + bias-gradient column sums) and every weight gradient
# (fp32 main_grad, split-K) run on the native MFMA kernels (csrc/gemm.hip); the plain projections
# (qkv / out / proj forward, qkv / out / fc dgrad) stay on the library GEMM, which the native kernel
# reaches only 0.83-0.93x of on those shapes (profiles/r3_gemm_lab.jsonl).
def _native_mlp(h2, wfc, bfc) -> bool:
    # the separate bias-GELU kernels remain only for shapes the native GEMM does not take (and the
    # CPU reference path)
    if not h2.is_cuda or bfc.dtype != torch.bfloat16:
        return False
    from . import gemm
    return gemm.supported(h2, wfc)


def _mm(a, b, bias=None):
    """a @ b (+ bias) on the library GEMM (plain projection)."""
    return torch.addmm(bias, a, b) if bias is not None else torch.mm(a, b)


def _native_env(name: str) -> bool:
    return os.environ.get(name, "0") == "1"


def _addmm_inplace(c, a, b):
    """c += a @ b (c is a fresh, un-saved buffer).  TDL_NATIVE_PROJ=1: the native kernel's
    residual-add epilogue instead of the library GEMM with beta = 1 (A/B switch)."""
    if c.is_cuda:
        if _native_env("TDL_NATIVE_PROJ"):
            from . import gemm
            if gemm.supported(a, b):
                return gemm.matmul(a, b, out=c, epi="resadd")
        return c.addmm_(a, b)
    return c.copy_((c.float() + a.float() @ b.float()).to(c.dtype))


# ---------------------------------------------------------------- the block
class _GPT2BlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ln1_w, ln1_b, w_qkv, b_qkv, w_o, b_o, ln2_w, ln2_b, w_fc, b_fc, w_p, b_p, n_head, eps):
        B, T, C = x.shape
        x2 = x.reshape(B * T, C)
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        h1, mean1, rstd1 = _ln_fwd(x2, ln1_w, ln1_b, eps)
        qkv = _mm(h1, fwd_weight(w_qkv), b_qkv)
        o, lse, scale = attn_fwd(qkv.view(B, T, 3 * C), n_head, True)
        o2 = o.view(B * T, C)
        if _native_env("TDL_NATIVE_OPROJ") and o2.is_cuda:   # A/B switch: native out-projection
            from . import gemm
            z = gemm.matmul(o2, fwd_weight(w_o))
        else:
            z = _mm(o2, fwd_weight(w_o))
        y1, y, h2, mean2, rstd2 = _add_bias_ln_fwd(x2, z, b_o, b_p, ln2_w, ln2_b, eps, (B, T, C))
        del z
        wfc = fwd_weight(w_fc)
        fused_mlp = _native_mlp(h2, wfc, b_fc)
        if fused_mlp:   # pre = h2 @ Wfc + bfc and f = gelu(pre) from one GEMM epilogue
            pre = torch.empty(h2.shape[0], wfc.shape[1], dtype=h2.dtype, device=h2.device)
            from . import gemm
            f = gemm.matmul(h2, wfc, bias=b_fc, epi="gelu", aux=pre)
        else:           # pre = h2 @ Wfc (bias added inside the GELU kernel)
            pre = torch.mm(h2, wfc)
            f = _bias_gelu_fwd(pre, b_fc)
        _addmm_inplace(y.view(B * T, C), f, fwd_weight(w_p))  # y = y1 + bp + f @ Wp
        ctx.save_for_backward(x2, h1, mean1, rstd1, qkv, o2, lse, y1, h2, mean2, rstd2, pre, f,
                              ln1_w, ln1_b, w_qkv, b_qkv, w_o, b_o, ln2_w, ln2_b, w_fc, b_fc, w_p, b_p)
        ctx.dims = (B, T, C, n_head, scale)
        ctx.fused_mlp = fused_mlp
        return y

    @staticmethod
    def backward(ctx, dy):
        (x2, h1, mean1, rstd1, qkv, o2, lse, y1, h2, mean2, rstd2, pre, f,
         ln1_w, ln1_b, w_qkv, b_qkv, w_o, b_o, ln2_w, ln2_b, w_fc, b_fc, w_p, b_p) = ctx.saved_tensors
        B, T, C, H, scale = ctx.dims
        params = (ln1_w, ln1_b, w_qkv, b_qkv, w_o, b_o, ln2_w, ln2_b, w_fc, b_fc, w_p, b_p)
        acc = [_f32_acc(p) for p in params]
        (g_ln1w, g_ln1b, g_wqkv, g_bqkv, g_wo, g_bo, g_ln2w, g_ln2b, g_wfc, g_bfc, g_wp, g_bp) = acc
        dy2 = dy.reshape(B * T, C)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        # weight-gradient GEMMs only accumulate into main_grad: queue them when the engine defers
        # them behind the input-gradient send (layers.defer_weight_grads); run inline otherwise
        wdefer = run_or_defer if all(_wants_main_grad(p) for p in (w_qkv, b_qkv, w_o, w_fc, w_p)) else (lambda fn: fn())
        # MLP branch
        sk = {id(g): take_stats_sink(g) for g in (g_wp, g_wfc, g_wo, g_wqkv)}   # verifier's fused reduces
        # the proj weight gradient goes with the fc one (one grouped launch) when both qualify
        pair_p = dy2.is_cuda and gemm_grouped_wgrad("mlp")
        if not pair_p:
            wdefer(lambda: wgrad_acc(g_wp, f.t(), dy2, sink=sk[id(g_wp)]))
        if ctx.fused_mlp and _native_mlp(dy2, w_p.t(), b_fc):
            from . import gemm   # dpre = (dy @ Wp^T) * gelu'(pre), bfc grad as column sums
            dpre = gemm.matmul(dy2, w_p.t(), epi="dgelu", aux=pre, colsum=g_bfc)
        else:
            df = torch.mm(dy2, w_p.t())
            if ctx.fused_mlp:    # pre already holds the bias
                dpre = _bias_gelu_bwd(df, pre, torch.zeros_like(b_fc), g_bfc)
            else:
                dpre = _bias_gelu_bwd(df, pre, b_fc, g_bfc)
            del df
        if pair_p:
            wdefer(lambda dpre=dpre: wgrad_acc_pair(g_wfc, h2.t(), dpre, g_wp, f.t(), dy2, sink1=sk[id(g_wfc)],
                                                    sink2=sk[id(g_wp)]))
        else:
            wdefer(lambda dpre=dpre: wgrad_acc(g_wfc, h2.t(), dpre, sink=sk[id(g_wfc)]))
        dh2 = _mm(dpre, w_fc.t())
        del dpre
        # dy1 = dy + LN2_bwd(dh2); bp grad = colsum(dy), bo grad = colsum(dy1) from the same pass
        dy1 = _ln_bwd(dh2, y1, ln2_w, mean2, rstd2, g_ln2w, g_ln2b, dres=dy2, sres_acc=g_bp, sdx_acc=g_bo)
        del dh2
        # attention branch
        # the o weight gradient goes with the qkv one (one grouped launch, wgrad_acc_pair) when both
        # qualify for it
        pair_o = dy1.is_cuda and gemm_grouped_wgrad("attn")
        if not pair_o:
            wdefer(lambda: wgrad_acc(g_wo, o2.t(), dy1, sink=sk[id(g_wo)]))
        do = _mm(dy1, w_o.t())
        # the qkv bias gradient (column sums of dqkv) comes out of the attention backward kernels
        dqkv = attn_bwd(qkv.view(B, T, 3 * C), o2.view(B, T, C), lse, do.view(B, T, C), H, True, scale,
                        bias_acc=g_bqkv)
        del do
        dqkv2 = dqkv.view(B * T, 3 * C)

        def _qkv_grads(dqkv2=dqkv2):
            if pair_o:
                wgrad_acc_pair(g_wqkv, h1.t(), dqkv2, g_wo, o2.t(), dy1, sink1=sk[id(g_wqkv)], sink2=sk[id(g_wo)])
            else:
                wgrad_acc(g_wqkv, h1.t(), dqkv2, sink=sk[id(g_wqkv)])
        wdefer(_qkv_grads)
        dx = None
        if ctx.needs_input_grad[0]:
            dh1 = _mm(dqkv2, w_qkv.t())
            dx = _ln_bwd(dh1, x2, ln1_w, mean1, rstd1, g_ln1w, g_ln1b, dres=dy1).view(B, T, C)
        grads = tuple(None if _wants_main_grad(p) else a.to(p.dtype) for p, a in zip(params, acc))
        return (dx, *grads, None, None)


def gpt2_block(x: torch.Tensor, blk) -> torch.Tensor:
    """Run a ``models.gpt2.GPT2Block`` (HF parameter layout) through the fused block."""
    a, m = blk.attn, blk.mlp
    return _GPT2BlockFn.apply(x, blk.ln_1.weight, blk.ln_1.bias, a.c_attn.weight, a.c_attn.bias,
                              a.c_proj.weight, a.c_proj.bias, blk.ln_2.weight, blk.ln_2.bias,
                              m.c_fc.weight, m.c_fc.bias, m.c_proj.weight, m.c_proj.bias, a.n_head, blk.ln_1.eps)
