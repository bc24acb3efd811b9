"""Autograd ops for the model compute path.

GPU tensors run the native gfx950 kernels (csrc/norm_act.hip, xent.hip, attention.hip, gemm.hip:
the weight-gradient products, the fused MLP GEMMs) and, for the plain bf16 projections where the
native GEMM is still slower, torch's hipBLASLt GEMM; CPU tensors run an equivalent PyTorch
reference, which is what the CPU/gloo tests exercise.

Gradient accumulation fusion: a parameter may carry ``.main_grad`` — an fp32 view into its
stage's flat gradient buffer (parallel/flat.py).  Ops then accumulate that parameter's
gradient straight into ``main_grad`` (fp32 atomics / beta=1 GEMM epilogue on GPU) and return
``None`` to autograd, so per-micro-batch bf16 weight-gradient tensors never exist.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import ptr, stream_ptr


def _accumulate(param: Optional[torch.Tensor], grad: Optional[torch.Tensor]):
    """Route a parameter gradient: into ``param.main_grad`` if present (returns None), else return it."""
    if param is None or grad is None:
        return None
    mg = getattr(param, "main_grad", None)
    if mg is None:
        return grad.to(param.dtype)
    if grad.is_cuda and grad.dtype != torch.float32 and grad.is_contiguous():
        _lib.call("tdl_add_into_f32", ptr(mg), ptr(grad), grad.numel(), 1, stream_ptr(grad.device))
    else:
        mg.add_(grad.reshape(mg.shape).float())
    return None


# ---------------------------------------------------------------- deferred weight gradients
# Inside ``defer_weight_grads()`` the fused backward ops queue their weight-gradient GEMMs (which
# only accumulate into fp32 ``main_grad``) instead of running them: the pipeline engine computes a
# stage's input gradient first, posts it to the previous stage, and only then runs the queued
# weight-gradient work while the transfer (and the upstream stage's backward) proceeds — the
# cooldown of a 1F1B schedule then advances one stage per B_input instead of per full backward
# (the B/W split of zero-bubble pipeline schedules).
_DEFER: Optional[list] = None


class defer_weight_grads:
    def __init__(self, enabled: bool = True):
        self.enabled = enabled
        self.pending: list = []

    def __enter__(self):
        global _DEFER
        self._prev = _DEFER
        if self.enabled:
            _DEFER = self.pending
        return self

    def __exit__(self, *exc):
        global _DEFER
        _DEFER = self._prev
        return False

    def run(self):
        pending, self.pending = self.pending, []
        for fn in pending:
            fn()


def run_or_defer(fn) -> None:
    if _DEFER is not None:
        _DEFER.append(fn)
    else:
        fn()


def _wants_main_grad(p: Optional[torch.Tensor]) -> bool:
    return p is not None and getattr(p, "main_grad", None) is not None


def _scratch(n: int, device) -> torch.Tensor:
    """fp32 workspace for per-block partial sums (stream-ordered caching allocator: free to reuse)."""
    return torch.empty(max(n, 1), dtype=torch.float32, device=device)


def _f32_acc(p: torch.Tensor) -> torch.Tensor:
    """fp32 buffer the kernels accumulate a param gradient into (main_grad or a fresh zero buffer)."""
    mg = getattr(p, "main_grad", None)
    return mg if mg is not None else torch.zeros(p.shape, dtype=torch.float32, device=p.device)


# ============================================================== LayerNorm
class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        M, N = x2.shape
        if x.is_cuda:
            y = torch.empty_like(x2)
            mean = torch.empty(M, dtype=torch.float32, device=x.device)
            rstd = torch.empty_like(mean)
            _lib.call("tdl_layernorm_fwd", ptr(x2), ptr(weight), ptr(bias), ptr(y), ptr(mean), ptr(rstd),
                      M, N, float(eps), stream_ptr(x.device))
        else:
            xf = x2.float()
            mean = xf.mean(-1)
            rstd = torch.rsqrt(xf.var(-1, unbiased=False) + eps)
            y = ((xf - mean[:, None]) * rstd[:, None] * weight.float() + bias.float()).to(x.dtype)
        ctx.save_for_backward(x2, weight, bias, mean, rstd)
        ctx.shape = shape
        return y.reshape(shape)

    @staticmethod
    def backward(ctx, dy):
        x2, weight, bias, mean, rstd = ctx.saved_tensors
        M, N = x2.shape
        dy2 = dy.reshape(M, N).contiguous()
        if dy.is_cuda:
            dx = torch.empty_like(x2)
            dw = _f32_acc(weight)
            db = _f32_acc(bias)
            _lib.call("tdl_layernorm_bwd", ptr(dy2), ptr(x2), ptr(weight), ptr(mean), ptr(rstd), ptr(dx),
                      ptr(dw), ptr(db), M, N, ptr(_scratch(2 * N * ((M + 7) // 8), dy.device)),
                      stream_ptr(dy.device))
            gw = None if _wants_main_grad(weight) else dw.to(weight.dtype)
            gb = None if _wants_main_grad(bias) else db.to(bias.dtype)
            return dx.reshape(ctx.shape), gw, gb, None
        xf, g = x2.float(), dy2.float()
        xh = (xf - mean[:, None]) * rstd[:, None]
        gw_ = g * weight.float()
        dx = rstd[:, None] * (gw_ - gw_.mean(-1, keepdim=True) - xh * (gw_ * xh).mean(-1, keepdim=True))
        return (dx.to(dy.dtype).reshape(ctx.shape), _accumulate(weight, (g * xh).sum(0)),
                _accumulate(bias, g.sum(0)), None)


def layer_norm(x, weight, bias, eps: float = 1e-5):
    return _LayerNorm.apply(x, weight, bias, eps)


# ============================================================== Linear (HF Conv1D layout: weight [in, out])
# ---------------------------------------------------------------- forward-layout weight copies
# hipBLASLt on gfx950 runs Y = X @ W fastest with W stored [out, in] (the "NT" form) and the input
# gradient dX = dY @ W^T fastest with W stored [in, out] (scripts/gemm_layout_probe.py,
# profiles/r1_gemm_layout_probe.jsonl: GPT-2-medium block shapes, 16k-32k tokens, forward
# +11-26 %, dgrad -12-16 % when the layout is swapped).  The parameters keep the HF [in, out]
# layout (checkpoints, dgrad); each forward GEMM reads a transposed bf16 copy that is rebuilt
# once per weight generation.  Generations advance on every optimizer update and at the start of
# every engine step (which covers re-shards, restores, checkpoint loads and injected parameter
# attacks); torch in-place writes are caught by the tensor version counter.
_WEIGHT_GEN = [0]


def bump_weight_generation() -> None:
    _WEIGHT_GEN[0] += 1


def _fwd_layout_enabled() -> bool:
    return os.environ.get("TDL_FWD_WEIGHT_T", "1") != "0"


def fwd_weight(w: torch.Tensor) -> torch.Tensor:
    """Operand for ``x @ W`` with W = ``w`` [in, out]: a view of a cached [out, in] copy on the
    GPU (same values, faster GEMM form), ``w`` itself elsewhere."""
    if not (w.is_cuda and w.dim() == 2 and _fwd_layout_enabled()):
        return w
    key = (_WEIGHT_GEN[0], w._version, w.data_ptr())
    cached = getattr(w, "_tdl_fwd_t", None)
    if cached is not None and cached[0] == key:
        return cached[1].t()
    if cached is not None and cached[1].shape == (w.shape[1], w.shape[0]) and cached[1].dtype == w.dtype:
        wt = cached[1]
    else:
        wt = torch.empty((w.shape[1], w.shape[0]), dtype=w.dtype, device=w.device)
    R, C = w.shape
    if w.dtype == torch.bfloat16 and w.is_contiguous() and R % 64 == 0 and C % 64 == 0:
        _lib.call("tdl_transpose_bf16", ptr(w), ptr(wt), R, C, stream_ptr(w.device))
    else:
        wt.copy_(w.t())
    w._tdl_fwd_t = (key, wt)
    return wt.t()


def prebuild_fwd_weights(weights) -> None:
    """Rebuild every stale forward-layout copy among ``weights`` (those ``fwd_weight`` has built
    before: the block projections and the tied LM-head weight) in batched native launches
    (tdl_transpose_bf16_batch, 64 weights per launch) instead of one launch per weight at its first
    use; the pipeline stage calls this at the head of each forward (parallel/stage.py).  Same copies
    and cache as ``fwd_weight``."""
    if not _fwd_layout_enabled():
        return
    todo = []
    for w in weights:
        cached = getattr(w, "_tdl_fwd_t", None)
        if cached is None or not w.is_cuda:
            continue
        key = (_WEIGHT_GEN[0], w._version, w.data_ptr())
        R, C = w.shape
        if (cached[0] != key and w.dtype == torch.bfloat16 and w.is_contiguous() and R % 64 == 0 and C % 64 == 0
                and cached[1].shape == (C, R)):
            todo.append((w, cached[1], key))
    for i in range(0, len(todo), _lib.TransposeBatch.MAX):
        chunk = todo[i:i + _lib.TransposeBatch.MAX]
        b = _lib.TransposeBatch()
        b.n = len(chunk)
        t = 0
        for j, (w, wt, key) in enumerate(chunk):
            R, C = w.shape
            b.inp[j], b.out[j], b.R[j], b.C[j], b.first[j] = w.data_ptr(), wt.data_ptr(), R, C, t
            t += (R // 64) * (C // 64)
            w._tdl_fwd_t = (key, wt)
        b.first[len(chunk)] = t
        _lib.call("tdl_transpose_bf16_batch", b, stream_ptr(chunk[0][0].device))


def _gemm_backend(t: torch.Tensor) -> str:
    return "gpu" if t.is_cuda else "cpu"


def _bias_grad_into(bias: torch.Tensor, dy2: torch.Tensor):
    """bias grad = column sums of dy2 [M, N] (bf16), accumulated in fp32 by one native pass."""
    if dy2.is_cuda and dy2.dtype == torch.bfloat16 and dy2.shape[1] % 8 == 0:
        acc = _f32_acc(bias)
        M, N = dy2.shape
        _lib.call("tdl_colsum_bf16", ptr(dy2), ptr(acc), M, N, ptr(_scratch(((M + 15) // 16) * N, dy2.device)),
                  stream_ptr(dy2.device))
        return None if _wants_main_grad(bias) else acc.to(bias.dtype)
    return _accumulate(bias, dy2.float().sum(0))


def take_stats_sink(acc: torch.Tensor):
    """The gradient verifier's fused-reduce hook armed on ``acc`` (a ``main_grad``) for this step's
    last accumulation, removed so it is used at most once.  Taken when the backward op runs (not
    when a deferred weight-gradient closure runs): backward order is micro-batch order."""
    sink = getattr(acc, "_tdl_stats_sink", None)
    if sink is not None:
        acc._tdl_stats_sink = None
    return sink


def wgrad_acc(acc: torch.Tensor, a: torch.Tensor, b: torch.Tensor, sink=None):
    """acc (fp32, shape of a @ b) += a @ b.

    ``a`` is usually X^T (a transposed view of a row-major [M, K] activation) and ``b`` dY: on the
    GPU the product runs on the native persistent 4-wave MFMA kernel (csrc/gemm.hip gemm_p4) with the
    token reduction split so the output tiles x slices fill the CUs in whole rounds, fp32 slices
    reduced into ``acc`` by one native pass (1.02-1.28x the hipBLASLt batched path on the GPT-2-medium
    weight gradients at 64k tokens: profiles/r3_gemm_lab.jsonl)."""
    if not a.is_cuda:
        acc.add_((a @ b).float().view(acc.shape))
        return
    from . import gemm
    if acc.dtype == torch.float32 and acc.is_contiguous() and acc.dim() == 2 and gemm.supported(a, b):
        gemm.matmul_f32_acc(acc, a, b, sink=sink)
        return
    # shapes the native kernel does not take (K % 64, unaligned rows): one library GEMM, fp32 out
    acc.add_(torch.mm(a, b, out_dtype=torch.float32).view(acc.shape))


def wgrad_acc_pair(acc1: torch.Tensor, a1: torch.Tensor, b1: torch.Tensor, acc2: torch.Tensor, a2: torch.Tensor,
                   b2: torch.Tensor, sink1=None, sink2=None):
    """Two weight gradients sharing K (tokens) — the attention's qkv and o, the MLP's fc and proj —
    from one grouped launch when they qualify (gemm.matmul_f32_acc_grouped), else one by one."""
    if a1.is_cuda:
        from . import gemm
        if gemm.matmul_f32_acc_grouped(acc1, a1, b1, acc2, a2, b2, sink1, sink2):
            return
    wgrad_acc(acc1, a1, b1, sink=sink1)
    wgrad_acc(acc2, a2, b2, sink=sink2)


def _wgrad_into(param: torch.Tensor, a: torch.Tensor, b: torch.Tensor):
    """param grad += a @ b, accumulating in fp32 into ``main_grad`` when present."""
    mg = getattr(param, "main_grad", None)
    if mg is None or not a.is_cuda:
        return _accumulate(param, a @ b)
    wgrad_acc(mg, a, b)
    return None


class _Linear(torch.autograd.Function):
    """y = x @ W + b with W stored [in, out] (HF GPT-2 Conv1D); ``act='gelu'`` fuses bias+GELU(tanh)."""

    @staticmethod
    def forward(ctx, x, weight, bias, act):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        backend = _gemm_backend(x)
        pre = None
        if backend == "cpu":
            y = x2 @ weight
            if bias is not None:
                y = y + bias
            if act == "gelu":
                pre = y
                y = F.gelu(y, approximate="tanh")
        else:  # torch GEMM + native bias-GELU kernel
            if act == "gelu":
                pre = torch.mm(x2, fwd_weight(weight))
                y = torch.empty_like(pre)
                _lib.call("tdl_bias_gelu_fwd", ptr(pre), ptr(bias), ptr(y), pre.shape[0], pre.shape[1],
                          stream_ptr(x.device))
            else:
                wf = fwd_weight(weight)
                y = torch.addmm(bias, x2, wf) if bias is not None else torch.mm(x2, wf)
        ctx.save_for_backward(x2, weight, bias, pre)
        ctx.act = act
        ctx.backend = backend
        ctx.shape = shape
        return y.reshape(*shape[:-1], weight.shape[1])

    @staticmethod
    def backward(ctx, dy):
        x2, weight, bias, pre = ctx.saved_tensors
        dy2 = dy.reshape(-1, weight.shape[1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        backend = ctx.backend
        if backend == "cpu":
            if ctx.act == "gelu":
                pre_ = pre.detach().requires_grad_(True)
                with torch.enable_grad():
                    out = F.gelu(pre_, approximate="tanh")
                dy2 = torch.autograd.grad(out, pre_, dy2)[0]
            dx = dy2 @ weight.t() if ctx.needs_input_grad[0] else None
            gw = _accumulate(weight, x2.t() @ dy2)
            gb = _accumulate(bias, dy2.sum(0)) if bias is not None else None
        else:
            if ctx.act == "gelu":
                dpre = torch.empty_like(pre)
                db = _f32_acc(bias)
                _lib.call("tdl_bias_gelu_bwd", ptr(dy2), ptr(pre), ptr(bias), ptr(dpre), ptr(db),
                          pre.shape[0], pre.shape[1],
                          ptr(_scratch(((pre.shape[0] + 15) // 16) * pre.shape[1], dy.device)), stream_ptr(dy.device))
                dy2 = dpre
                gb = None if _wants_main_grad(bias) else db.to(bias.dtype)
            else:
                gb = _bias_grad_into(bias, dy2) if bias is not None else None
            dx = torch.mm(dy2, weight.t()) if ctx.needs_input_grad[0] else None
            gw = _wgrad_into(weight, x2.t(), dy2)
        if dx is not None:
            dx = dx.reshape(ctx.shape)
        return dx, gw, gb, None


def linear(x, weight, bias=None, act: Optional[str] = None):
    return _Linear.apply(x, weight, bias, act)


# ============================================================== causal self-attention on packed qkv
def attn_fwd(qkv: torch.Tensor, n_head: int, causal: bool):
    """qkv [B, T, 3*H*D] (contiguous) -> (out [B, T, H*D], lse [B*H, T] fp32, scale)."""
    B, T, C3 = qkv.shape
    D = C3 // (3 * n_head)
    scale = 1.0 / math.sqrt(D)
    if qkv.is_cuda:
        if D != 64 or T % 128 != 0:
            raise ValueError(f"native attention supports head_dim 64 and T % 128 == 0 (got D={D}, T={T})")
        out = torch.empty(B, T, n_head * D, dtype=qkv.dtype, device=qkv.device)
        lse = torch.empty(B * n_head, T, dtype=torch.float32, device=qkv.device)
        _lib.call("tdl_attn_fwd", ptr(qkv), ptr(out), ptr(lse), None, B, T, n_head, D, scale, int(causal),
                  stream_ptr(qkv.device))
        return out, lse, scale
    q, k, v = qkv.float().view(B, T, 3, n_head, D).permute(2, 0, 3, 1, 4)
    att = (q @ k.transpose(-1, -2)) * scale
    if causal:
        att = att.masked_fill(torch.ones(T, T, dtype=torch.bool).triu(1), float("-inf"))
    lse = torch.logsumexp(att, -1).reshape(B * n_head, T)
    out = (torch.softmax(att, -1) @ v).transpose(1, 2).reshape(B, T, n_head * D).to(qkv.dtype)
    return out, lse, scale


def attn_bwd(qkv, out, lse, dout, n_head: int, causal: bool, scale: float,
             bias_acc: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Gradient w.r.t. the packed qkv (same layout as ``qkv``).  ``bias_acc`` (fp32 [3 H D]): the
    qkv bias gradient (column sums of the returned gradient) is accumulated into it — on the GPU
    from inside the two backward kernels (no pass over the [tokens, 3 H D] gradient)."""
    B, T, C3 = qkv.shape
    H = n_head
    D = C3 // (3 * H)
    dout = dout.contiguous()
    if qkv.is_cuda:
        dqkv = torch.empty_like(qkv)
        delta = torch.empty(B * H, T, dtype=torch.float32, device=qkv.device)
        part = None
        if bias_acc is not None:
            part = _scratch(B * (T // 128) * 3 * H * D, qkv.device)
        _lib.call("tdl_attn_bwd", ptr(qkv), ptr(out), ptr(dout), ptr(lse), ptr(dqkv), ptr(bias_acc), ptr(part),
                  ptr(delta), B, T, H, D, scale, int(causal), stream_ptr(qkv.device))
        return dqkv
    with torch.enable_grad():
        x = qkv.detach().float().requires_grad_(True)
        q, k, v = x.view(B, T, 3, H, D).permute(2, 0, 3, 1, 4)
        att = (q @ k.transpose(-1, -2)) * scale
        if causal:
            att = att.masked_fill(torch.ones(T, T, dtype=torch.bool).triu(1), float("-inf"))
        o = (torch.softmax(att, -1) @ v).transpose(1, 2).reshape(B, T, H * D)
        (g,) = torch.autograd.grad(o, x, dout.reshape(o.shape).float())
    g = g.to(qkv.dtype)
    if bias_acc is not None:
        bias_acc.add_(g.float().reshape(-1, C3).sum(0))
    return g


class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, n_head, causal):
        qkv = qkv.contiguous()
        out, lse, scale = attn_fwd(qkv, n_head, causal)
        ctx.save_for_backward(qkv, out, lse)
        ctx.n_head, ctx.causal, ctx.scale = n_head, causal, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        return attn_bwd(qkv, out, lse, dout, ctx.n_head, ctx.causal, ctx.scale), None, None


def causal_attention(qkv: torch.Tensor, n_head: int, causal: bool = True) -> torch.Tensor:
    """qkv: [B, T, 3*H*D] packed (c_attn output) -> [B, T, H*D]."""
    return _Attention.apply(qkv, n_head, causal)


# ============================================================== token + position embedding
class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, wte, wpe):
        B, T = ids.shape
        H = wte.shape[1]
        ids = ids.contiguous()
        if ids.is_cuda:
            out = torch.empty(B, T, H, dtype=wte.dtype, device=wte.device)
            _lib.call("tdl_embedding_fwd", ptr(ids), ptr(wte), ptr(wpe), ptr(out), B, T, H, 0,
                      stream_ptr(ids.device))
        else:
            out = wte[ids] + wpe[:T].unsqueeze(0)
        ctx.save_for_backward(ids, wte, wpe)
        return out

    @staticmethod
    def backward(ctx, dout):
        ids, wte, wpe = ctx.saved_tensors
        B, T = ids.shape
        H = wte.shape[1]
        dout = dout.contiguous()
        if dout.is_cuda:
            gte = _f32_acc(wte)
            gpe = _f32_acc(wpe)
            _lib.call("tdl_embedding_bwd", ptr(ids), ptr(dout), ptr(gte), ptr(gpe), B, T, H, 0,
                      stream_ptr(dout.device))
            return (None, None if _wants_main_grad(wte) else gte.to(wte.dtype),
                    None if _wants_main_grad(wpe) else gpe.to(wpe.dtype))
        gte = torch.zeros(wte.shape, dtype=torch.float32)
        gte.index_add_(0, ids.reshape(-1), dout.reshape(-1, H).float())
        gpe = torch.zeros(wpe.shape, dtype=torch.float32)
        gpe[:T] = dout.float().sum(0)
        return None, _accumulate(wte, gte), _accumulate(wpe, gpe)


def embedding(ids, wte, wpe):
    return _Embedding.apply(ids, wte, wpe)


# ============================================================== softmax cross-entropy (padded vocab aware)
class _CrossEntropy(torch.autograd.Function):
    """Mean CE over rows of logits [M, ld] whose first ``V`` columns are real classes."""

    @staticmethod
    def forward(ctx, logits, labels, V):
        M, ld = logits.shape
        labels = labels.reshape(-1).contiguous()
        if logits.is_cuda:
            loss_rows = torch.empty(M, dtype=torch.float32, device=logits.device)
            lse = torch.empty(M, dtype=torch.float32, device=logits.device)
            _lib.call("tdl_xent_fwd", ptr(logits), ptr(labels), ptr(loss_rows), ptr(lse), M, V, ld,
                      stream_ptr(logits.device))
        else:
            lf = logits[:, :V].float()
            lse = torch.logsumexp(lf, -1)
            valid = labels >= 0
            picked = lf.gather(1, labels.clamp(min=0)[:, None])[:, 0]
            loss_rows = torch.where(valid, lse - picked, torch.zeros_like(lse))
        n_valid = (labels >= 0).sum().clamp(min=1).float()
        ctx.save_for_backward(logits, labels, lse, n_valid)
        ctx.V = V
        return loss_rows.sum() / n_valid

    @staticmethod
    def backward(ctx, g):
        logits, labels, lse, n_valid = ctx.saved_tensors
        M, ld = logits.shape
        V = ctx.V
        scale = (g.float() / n_valid).reshape(1).contiguous()
        if logits.is_cuda:
            # in place: the logits buffer is dead once the loss has been taken
            _lib.call("tdl_xent_bwd", ptr(logits), ptr(labels), ptr(lse), ptr(scale), ptr(logits), M, V, ld, 0.0,
                      stream_ptr(logits.device))
            return logits, None, None
        p = torch.exp(logits.float() - lse[:, None])
        p[:, V:] = 0.0
        valid = labels >= 0
        p[torch.arange(M)[valid], labels[valid]] -= 1.0
        p = p * valid[:, None].float() * scale
        return p.to(logits.dtype), None, None


def cross_entropy(logits, labels, num_classes: Optional[int] = None):
    V = logits.shape[-1] if num_classes is None else num_classes
    return _CrossEntropy.apply(logits.reshape(-1, logits.shape[-1]), labels, V)


# ============================================================== Linear with nn.Linear weight layout [out, in]
class _LinearT(torch.autograd.Function):
    """y = x @ W^T, W stored [out, in] (used by the tied LM head: W = wte [vocab, n_embd])."""

    @staticmethod
    def forward(ctx, x, weight):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        backend = _gemm_backend(x)
        if backend == "cpu":
            y = x2 @ weight.t()
        else:
            y = torch.mm(x2, weight.t())
        ctx.save_for_backward(x2, weight)
        ctx.backend, ctx.shape = backend, shape
        return y.reshape(*shape[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, weight = ctx.saved_tensors
        dy2 = dy.reshape(-1, weight.shape[0])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = (dy2 @ weight) if ctx.needs_input_grad[0] else None
        if _wants_main_grad(weight):
            run_or_defer(lambda: _wgrad_into(weight, dy2.t(), x2))
            gw = None
        else:
            gw = _wgrad_into(weight, dy2.t(), x2)
        return (dx.reshape(ctx.shape) if dx is not None else None), gw


def linear_t(x, weight):
    return _LinearT.apply(x, weight)


# ============================================================== tied LM head + cross-entropy, one node
def lmhead_chunk_rows(vocab_padded: int) -> int:
    """Rows per logits chunk: the whole micro-batch unless its bf16 logits exceed
    TDL_LMHEAD_CHUNK_MB (default 8192 MB) — then the [rows, vocab] logits are never materialised
    at once."""
    budget = int(os.environ.get("TDL_LMHEAD_CHUNK_MB", "8192")) << 20
    return max(256, budget // (2 * vocab_padded) // 256 * 256)


def _scale_bf16(x: torch.Tensor, y: torch.Tensor, g: torch.Tensor):
    """y = x * g[0] (g: fp32 device scalar; one rounding, no host sync)."""
    if x.dtype == torch.bfloat16 and x.numel() % 8 == 0 and x.is_contiguous() and y.is_contiguous():
        _lib.call("tdl_scale_bf16", ptr(x), ptr(y), ptr(g), x.numel(), stream_ptr(x.device))
    else:
        torch.mul(x, g.reshape(()), out=y)


def _lmhead_dx(dl: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """dX = dL @ W (W = wte [Vp, n]) on the persistent LDS-DMA kernel (gemm_pd) over a [n, Vp] copy
    of W (``fwd_weight``: one native transpose per weight generation, ~30 us): the NT form of the
    product runs 4565 vs 5004 us for the library's at the bench shape (profiles/r6_lmhead_ab.jsonl).
    ``TDL_LMHEAD_DX=lib`` keeps the library GEMM (A/B switch)."""
    from . import gemm
    if os.environ.get("TDL_LMHEAD_DX", "pd") == "pd" and dl.is_cuda:
        wt = fwd_weight(weight)       # logical [Vp, n], stored [n][Vp]: k-contiguous
        if gemm.supported(dl, wt):
            return gemm.matmul(dl, wt, kernel="pd")
    return torch.mm(dl, weight)


class _LMHeadXent(torch.autograd.Function):
    """loss = mean CE(x @ W^T, labels) with W = wte [Vp, n] tied; padded vocab columns masked.

    The CE forward and backward run as ONE native pass per logits row (tdl_xent_fused: loss,
    log-sum-exp, then dlogits = (softmax - onehot) / n_valid written over the logits in place),
    during the forward: the logits are read + written once.  ``observe(logits)`` (the stage's
    output monitor) runs before the overwrite.  One chunk (the usual case): the dlogits buffer is
    kept and the backward runs dX = g dL.W and dW += dL^T.(g X) (deferrable with the B/W split).
    Several chunks (logits above the budget): each chunk's dX / dW are formed right away into
    fp32 buffers that the backward scales by the upstream gradient g."""

    @staticmethod
    def forward(ctx, x, weight, labels, V, observe, chunk_rows):
        shape = x.shape
        n = shape[-1]
        x2 = x.reshape(-1, n).contiguous()
        N, Vp = x2.shape[0], weight.shape[0]
        labels = labels.reshape(-1).contiguous()
        dev = x2.device
        n_valid = ((labels >= 0) & (labels < V)).sum().clamp(min=1).float()
        scale = (1.0 / n_valid).reshape(1).contiguous()
        loss_rows = torch.empty(N, dtype=torch.float32, device=dev)
        lse = torch.empty(N, dtype=torch.float32, device=dev)
        s = stream_ptr(dev)
        C = N if chunk_rows is None or chunk_rows >= N else int(chunk_rows)
        ctx.shape = shape
        if C == N:
            logits = torch.mm(x2, weight.t())
            if observe is not None:
                observe(logits)
            _lib.call("tdl_xent_fused", ptr(logits), ptr(labels), ptr(loss_rows), ptr(lse), ptr(scale), N, V, Vp, s)
            ctx.save_for_backward(x2, weight, logits)  # logits buffer now holds dL (unscaled by g)
            ctx.chunked = False
        else:
            dx = torch.empty(N, n, dtype=torch.float32, device=dev)
            dw = torch.zeros(Vp, n, dtype=torch.float32, device=dev)
            buf = torch.empty(C, Vp, dtype=x2.dtype, device=dev)
            for r0 in range(0, N, C):
                r1 = min(N, r0 + C)
                lc = buf[: r1 - r0]
                torch.mm(x2[r0:r1], weight.t(), out=lc)
                if observe is not None and r0 == 0:
                    observe(lc)
                _lib.call("tdl_xent_fused", ptr(lc), ptr(labels[r0:r1]), ptr(loss_rows[r0:r1]), ptr(lse[r0:r1]),
                          ptr(scale), r1 - r0, V, Vp, s)
                torch.mm(lc, weight, out_dtype=torch.float32, out=dx[r0:r1])
                wgrad_acc(dw, lc.t(), x2[r0:r1])
            ctx.save_for_backward(dx, dw, weight)
            ctx.chunked = True
        return loss_rows.sum() / n_valid

    @staticmethod
    def backward(ctx, g):
        g = g.reshape(())
        if ctx.chunked:
            dx32, dw, weight = ctx.saved_tensors
            dx = (dx32 * g).to(weight.dtype) if ctx.needs_input_grad[0] else None
            mg = getattr(weight, "main_grad", None)
            if mg is not None:
                mg.add_(dw * g)
                gw = None
            else:
                gw = (dw * g).to(weight.dtype)
        else:
            x2, weight, dl = ctx.saved_tensors
            gf = g.float().reshape(1).contiguous()
            dx = None
            if ctx.needs_input_grad[0]:
                dx = _lmhead_dx(dl, weight)
                _scale_bf16(dx, dx, gf)
            xg = torch.empty_like(x2)
            _scale_bf16(x2, xg, gf)
            if _wants_main_grad(weight):
                run_or_defer(lambda: _wgrad_into(weight, dl.t(), xg))
                gw = None
            else:
                gw = _wgrad_into(weight, dl.t(), xg)
        return (dx.reshape(ctx.shape) if dx is not None else None), gw, None, None, None, None


def lm_head_cross_entropy(x, weight, labels, num_classes: int, observe=None, chunk_rows: Optional[int] = None):
    """Mean CE of the tied LM head ``x @ weight^T`` (GPU: fused single-pass CE, chunked logits;
    CPU / no-grad: plain logits + cross_entropy).  ``observe`` sees the logits before reuse."""
    fused = os.environ.get("TDL_FUSED_LMHEAD", "1") != "0"
    if not (fused and x.is_cuda and torch.is_grad_enabled() and (x.requires_grad or weight.requires_grad)):
        logits = linear_t(x, weight)
        if observe is not None:
            observe(logits)
        return cross_entropy(logits.reshape(-1, logits.shape[-1]), labels.reshape(-1), num_classes)
    if chunk_rows is None:
        chunk_rows = lmhead_chunk_rows(weight.shape[0])
    return _LMHeadXent.apply(x, weight, labels, num_classes, observe, chunk_rows)
