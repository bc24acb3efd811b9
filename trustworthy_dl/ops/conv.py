"""Convolution + BatchNorm (+ residual) (+ ReLU) blocks for VGG / ResNet stages.

GPU bf16 tensors run the native gfx950 kernels — implicit-GEMM MFMA convolutions
(csrc/conv.hip: forward with fused per-channel batch statistics, data gradient, weight gradient
accumulated into the parameter's fp32 ``main_grad``) and one-pass NHWC BatchNorm/residual/ReLU
(csrc/bn.hip).  Activations are NHWC (torch ``channels_last``); weights keep the nn.Conv2d
[Cout, Cin, R, S] parameter layout (so state dicts / checkpoints are unchanged) and are permuted
to the kernel's [Cout][R][S][Cin] once per call (a weight-sized copy, tiny next to the GEMM).
Input channel counts that are not a multiple of 8 (the 3-channel image stem) are zero-padded to 8.

CPU (and fp32) tensors run the PyTorch modules themselves — the reference semantics the CPU/gloo
tests and the layer-cost hooks see.  There is no silent fallback on a GPU: a bf16 CUDA conv that
the kernels cannot serve raises.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib
from ._lib import ptr, stream_ptr
from .layers import _scratch
from .side_stream import WgradSide, wait_wgrad  # noqa: F401  (wait_wgrad: re-exported)

_NUM_CU = {}


def _num_cu(dev: torch.device) -> int:
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    n = _NUM_CU.get(idx)
    if n is None:
        n = torch.cuda.get_device_properties(idx).multi_processor_count
        _NUM_CU[idx] = n
    return n


def _wgrad(dev: torch.device, fn, keep):
    if WgradSide.on("TDL_CONV_WGRAD_SIDE", "1") and not torch.is_grad_enabled():
        WgradSide.run(dev, fn, keep)
    else:
        fn()


def _conv_ws(M: int, Cout: int, K: int, parity: bool, dev) -> torch.Tensor:
    """Workspace of one tdl_conv_nt* call: statistics partial rows + finalize counters, and the
    split-K slices when the kernel splits the reduction (csrc/conv.hip conv_split_of)."""
    return torch.empty(int(_lib.lib().tdl_conv_ws_floats(M, Cout, K, int(parity))), dtype=torch.float32, device=dev)


def _conv_fwd_bn(bnfin: dict, act, wk, out, stats, ws, dims, pro, dev) -> None:
    """Forward convolution whose output's BatchNorm (``bnfin["bn"]``, folded into the next
    convolution) is finalized by the convolution's own finishing workgroups (csrc/conv.hip BnFin):
    fills bnfin with the BN's [scale | shift | mean | rstd] buffer, its zeroed backward-sum row and
    ``done`` (False: the consumer runs tdl_bn_finalize itself)."""
    import ctypes
    bn = bnfin["bn"]
    Cout, M = dims[6], dims[0] * dims[4] * dims[5]   # dims = (N, H, W, C, P, Q, Cout, R, S, stride, pad)
    bnp = torch.empty(4 * Cout, dtype=torch.float32, device=dev)
    sums = torch.empty(int(_lib.lib().tdl_bn_bwd_ws_floats(Cout)), dtype=torch.float32, device=dev)
    upd = bn.running_mean is not None
    b = _lib.BnFin(bn.weight.data_ptr(), bn.bias.data_ptr(), bnp[2 * Cout:].data_ptr(), bnp[3 * Cout:].data_ptr(),
                   bn.running_mean.data_ptr() if upd else None, bn.running_var.data_ptr() if upd else None,
                   bnp.data_ptr(), sums.data_ptr(), M, float(bn.eps),
                   float(bn.momentum if bn.momentum is not None else 0.1))
    done = ctypes.c_int(0)
    _lib.call("tdl_conv_fwd_bn", ptr(act), ptr(wk), ptr(out), ptr(stats), ptr(ws), *dims, ptr(pro), ctypes.byref(b),
              ctypes.byref(done), stream_ptr(dev))
    bnfin.update(bnp=bnp, sums=sums, done=bool(done.value))


def native_conv_ok(x: torch.Tensor) -> bool:
    return x.is_cuda and x.dtype == torch.bfloat16


def _out_hw(H: int, W: int, R: int, S: int, stride: int, pad: int):
    return (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1


def _weight_layout(weight: torch.Tensor, cp: int, kind: str) -> torch.Tensor:
    """The kernel layouts of a conv weight [Cout, C, R, S]: ``"krsc"`` = [Cout][R][S][cp] (forward),
    ``"crsk"`` = [cp][R][S][Cout] (data gradient), input channels zero-padded to ``cp``.  Both are
    built by one native pass (tdl_conv_weight_layouts) the first time either is asked for in a weight
    generation (every optimizer update / engine step bumps it, in-place torch writes bump the tensor
    version: ops/layers.py fwd_weight) and cached on the parameter, so the forward, the backward and
    later micro-batches share them."""
    from .layers import _WEIGHT_GEN
    key = (_WEIGHT_GEN[0], weight._version, weight.data_ptr(), cp)
    hit = getattr(weight, "_tdl_conv_layouts", None)
    if hit is None or hit[0] != key:
        Cout, C, R, S = weight.shape
        if weight.is_cuda and weight.dtype == torch.bfloat16 and weight.is_contiguous():
            krsc = torch.empty((Cout, R, S, cp), dtype=weight.dtype, device=weight.device)
            crsk = torch.empty((cp, R, S, Cout), dtype=weight.dtype, device=weight.device)
            _lib.call("tdl_conv_weight_layouts", ptr(weight), ptr(krsc), ptr(crsk), Cout, C, cp, R * S,
                      stream_ptr(weight.device))
        else:
            wp = weight
            if cp != C:
                wp = torch.zeros((Cout, cp, R, S), dtype=weight.dtype, device=weight.device)
                wp[:, :C].copy_(weight)
            krsc, crsk = wp.permute(0, 2, 3, 1).contiguous(), wp.permute(1, 2, 3, 0).contiguous()
        hit = (key, {"krsc": krsc, "crsk": crsk})
        try:
            weight._tdl_conv_layouts = hit
        except (AttributeError, RuntimeError):
            pass
    return hit[1][kind]


def prebuild_layouts(weights) -> None:
    """Build the kernel layouts of every conv weight in ``weights`` whose cached layouts are stale
    (a new weight generation) in batched native launches (tdl_conv_weight_layouts_batch, 32
    weights per launch) instead of one launch per weight at its first use: the pipeline stage calls
    this at the head of each forward (parallel/stage.py).  Same outputs and cache as _weight_layout."""
    from .layers import _WEIGHT_GEN
    todo = []
    for w in weights:
        if not (w.is_cuda and w.dtype == torch.bfloat16 and w.is_contiguous() and w.dim() == 4):
            continue
        cp = (w.shape[1] + 7) // 8 * 8
        key = (_WEIGHT_GEN[0], w._version, w.data_ptr(), cp)
        hit = getattr(w, "_tdl_conv_layouts", None)
        if hit is None or hit[0] != key:
            todo.append((w, cp, key))
    for i in range(0, len(todo), _lib.LayoutBatch.MAX):
        chunk = todo[i:i + _lib.LayoutBatch.MAX]
        b = _lib.LayoutBatch()
        b.n = len(chunk)
        for j, (w, cp, key) in enumerate(chunk):
            Cout, C, R, S = w.shape
            krsc = torch.empty((Cout, R, S, cp), dtype=w.dtype, device=w.device)
            crsk = torch.empty((cp, R, S, Cout), dtype=w.dtype, device=w.device)
            b.w[j], b.krsc[j], b.crsk[j] = w.data_ptr(), krsc.data_ptr(), crsk.data_ptr()
            b.Cout[j], b.C[j], b.Cp[j], b.RS[j] = Cout, C, cp, R * S
            try:
                w._tdl_conv_layouts = (key, {"krsc": krsc, "crsk": crsk})
            except (AttributeError, RuntimeError):
                pass
        _lib.call("tdl_conv_weight_layouts_batch", b, stream_ptr(chunk[0][0].device))


def _pad_channels(x: torch.Tensor, cp: int) -> torch.Tensor:
    N, C, H, W = x.shape
    xp = torch.empty((N, cp, H, W), dtype=x.dtype, device=x.device, memory_format=torch.channels_last).zero_()
    xp[:, :C].copy_(x)
    return xp


class _Conv2dNHWC(torch.autograd.Function):
    """y = conv2d(x, w) on NHWC bf16; also returns per-channel (sum, sumsq) of y when asked."""

    @staticmethod
    def forward(ctx, x, weight, stride: int, pad: int, want_stats: bool, bnfin=None):
        N, C, H, W = x.shape
        Cout, Cw, R, S = weight.shape
        if Cw != C or Cout % 8 != 0:
            raise ValueError(f"native conv: unsupported shapes x={tuple(x.shape)} w={tuple(weight.shape)}")
        cp = (C + 7) // 8 * 8
        xs = x.contiguous(memory_format=torch.channels_last)
        if cp != C:
            xs = _pad_channels(xs, cp)
        wk = _weight_layout(weight, cp, "krsc")
        P, Q = _out_hw(H, W, R, S, stride, pad)
        y = torch.empty((N, Cout, P, Q), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        stats = None
        if want_stats:
            stats = torch.empty(2 * Cout, dtype=torch.float32, device=x.device)
        ws = _conv_ws(N * P * Q, Cout, R * S * cp, False, x.device)
        if want_stats and bnfin is not None:
            _conv_fwd_bn(bnfin, xs, wk, y, stats, ws, (N, H, W, cp, P, Q, Cout, R, S, stride, pad), None, x.device)
        else:
            _lib.call("tdl_conv_nt", ptr(xs), ptr(wk), ptr(y), ptr(stats), ptr(ws), N, H, W, cp, P, Q, Cout, R, S,
                      stride, pad, 0, stream_ptr(x.device))
        ctx.save_for_backward(xs, weight)
        ctx.geom = (N, C, cp, H, W, Cout, R, S, P, Q, stride, pad)
        # the statistics output never gets a gradient: without this autograd launches a zero fill
        # for it in every backward (one per convolution per step)
        ctx.set_materialize_grads(False)
        if stats is None:
            stats = torch.zeros(0, dtype=torch.float32, device=x.device)
        ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        if dy is None:
            return None, None, None, None, None, None
        xs, weight = ctx.saved_tensors
        N, C, cp, H, W, Cout, R, S, P, Q, stride, pad = ctx.geom
        dy = dy.contiguous(memory_format=torch.channels_last)
        if dy.dtype != xs.dtype:
            dy = dy.to(xs.dtype)
        dev = dy.device
        dx = None
        if ctx.needs_input_grad[0]:
            wd = _weight_layout(weight, cp, "crsk")  # [cp][R][S][Cout]
            dxp = torch.empty((N, cp, H, W), dtype=dy.dtype, device=dev, memory_format=torch.channels_last)
            wsd = _conv_ws(N * H * W, cp, R * S * Cout, stride == 2, dev)
            _lib.call("tdl_conv_nt", ptr(dy), ptr(wd), ptr(dxp), None, ptr(wsd), N, P, Q, Cout, H, W, cp, R, S, stride,
                      pad, 1, stream_ptr(dev))
            dx = dxp if cp == C else dxp[:, :C]
        gw = None
        if ctx.needs_input_grad[1]:
            mg = getattr(weight, "main_grad", None)
            if mg is not None and cp == C and mg.is_contiguous():
                # into the fp32 main_grad: on the weight-gradient stream, beside the data gradient
                ws = torch.empty(Cout * R * S * cp, dtype=torch.float32, device=dev) if R * S > 1 else None
                _wgrad(dev, lambda: _lib.call("tdl_conv_wgrad", ptr(dy), ptr(xs), ptr(mg), ptr(ws), N, H, W, cp, P, Q,
                                              Cout, R, S, stride, pad, _num_cu(dev), stream_ptr(dev)), (dy, xs, ws))
            else:
                acc = torch.zeros((Cout, cp, R, S), dtype=torch.float32, device=dev)
                ws = torch.empty(Cout * R * S * cp, dtype=torch.float32, device=dev) if R * S > 1 else None
                _lib.call("tdl_conv_wgrad", ptr(dy), ptr(xs), ptr(acc), ptr(ws), N, H, W, cp, P, Q, Cout, R, S, stride,
                          pad, _num_cu(dev), stream_ptr(dev))
                g = acc if cp == C else acc[:, :C]
                if mg is not None:
                    mg.add_(g)
                else:
                    gw = g.to(weight.dtype)
        return dx, gw, None, None, None, None


class _BatchNormActNHWC(torch.autograd.Function):
    """out = act(BN(y) (+ residual)) with batch statistics (training) from the conv epilogue."""

    @staticmethod
    def forward(ctx, y, stats, gamma, beta, residual, running_mean, running_var, training: bool,
                momentum: float, eps: float, relu: bool):
        N, C, H, W = y.shape
        M = N * H * W
        y = y.contiguous(memory_format=torch.channels_last)
        res = None
        if residual is not None:
            res = residual.contiguous(memory_format=torch.channels_last)
            if res.dtype != y.dtype:
                res = res.to(y.dtype)
        out = torch.empty_like(y, memory_format=torch.channels_last)
        mean = torch.empty(C, dtype=torch.float32, device=y.device)
        rstd = torch.empty_like(mean)
        upd = training and running_mean is not None
        # the backward's replicated reduction buffer, zeroed by this forward kernel
        ws = torch.empty(int(_lib.lib().tdl_bn_bwd_ws_floats(C)), dtype=torch.float32, device=y.device) \
            if training else None
        _lib.call("tdl_bn_act_fwd", ptr(y), ptr(stats if training else None), ptr(running_mean), ptr(running_var),
                  ptr(gamma), ptr(beta), ptr(res), ptr(out), ptr(mean), ptr(rstd),
                  ptr(running_mean if upd else None), ptr(running_var if upd else None), ptr(ws), M, C, float(eps),
                  float(momentum), int(relu), stream_ptr(y.device))
        ctx.ws = ws
        ctx.save_for_backward(y, out, mean, rstd, gamma, beta)
        ctx.cfg = (M, C, relu, residual is not None, training)
        return out

    @staticmethod
    def backward(ctx, dout):
        y, out, mean, rstd, gamma, beta = ctx.saved_tensors
        M, C, relu, has_res, training = ctx.cfg
        if not training:
            raise RuntimeError("native BatchNorm backward requires training mode (batch statistics)")
        dev = dout.device
        dout = dout.contiguous(memory_format=torch.channels_last)
        if dout.dtype != y.dtype:
            dout = dout.to(y.dtype)
        dx = torch.empty_like(y, memory_format=torch.channels_last)
        dres = torch.empty_like(y, memory_format=torch.channels_last) if has_res else None
        sums = ctx.ws
        mg_g, mg_b = getattr(gamma, "main_grad", None), getattr(beta, "main_grad", None)
        dg = mg_g if mg_g is not None else torch.zeros(C, dtype=torch.float32, device=dev)
        db = mg_b if mg_b is not None else torch.zeros(C, dtype=torch.float32, device=dev)
        # the per-block partial rows are scratch of this call only (not kept from the forward)
        part = _scratch(int(_lib.lib().tdl_bn_bwd_part_floats(C)), dev)
        _lib.call("tdl_bn_act_bwd", ptr(dout), ptr(out), ptr(y), ptr(mean), ptr(rstd), ptr(gamma), ptr(sums), ptr(part), ptr(dx),
                  ptr(dres), ptr(dg), ptr(db), M, C, int(relu), stream_ptr(dev))
        gg = None if mg_g is not None else dg.to(gamma.dtype)
        gb = None if mg_b is not None else db.to(beta.dtype)
        return dx, None, gg, gb, dres, None, None, None, None, None, None


class _BNActConvNHWC(torch.autograd.Function):
    """y_next = conv(relu(BN(y)), w) with the BN output never materialised: the batch statistics
    of y (from the producing conv's epilogue) are folded into a per-channel scale / shift
    (tdl_bn_finalize, no pass over y), the forward conv applies relu(y * scale + shift) while it
    stages its activation operand, the weight gradient re-applies it on its own load, and the BN
    backward recomputes the ReLU mask from y (tdl_bn_act_bwd_pro).  Saves the BN-apply pass, the
    write of its output and every later read of it (training mode only)."""

    @staticmethod
    def forward(ctx, y, stats, gamma, beta, running_mean, running_var, momentum: float, eps: float, weight,
                stride: int, pad: int, want_stats: bool, pre=None, bnfin=None):
        N, C, H, W = y.shape
        Cout, Cw, R, S = weight.shape
        if Cw != C or C % 8 or Cout % 8:
            raise ValueError(f"folded BN conv: unsupported shapes y={tuple(y.shape)} w={tuple(weight.shape)}")
        dev = y.device
        ys = y.contiguous(memory_format=torch.channels_last)
        M = N * H * W
        # [scale | shift | mean | rstd] in one buffer: the backward's data-gradient epilogue reads all four
        # pre: this BN already finalized by the producing convolution (_conv_fwd_bn)
        if pre is not None and "bnp" in pre:
            bnp, sums = pre["bnp"], pre["sums"]
        else:
            bnp = torch.empty(4 * C, dtype=torch.float32, device=dev)
            sums = torch.empty(int(_lib.lib().tdl_bn_bwd_ws_floats(C)), dtype=torch.float32, device=dev)
        pro, mean, rstd = bnp[:2 * C], bnp[2 * C:3 * C], bnp[3 * C:]
        upd = running_mean is not None
        if not (pre is not None and pre.get("done")):
            _lib.call("tdl_bn_finalize", ptr(stats), ptr(gamma), ptr(beta), ptr(mean), ptr(rstd),
                      ptr(running_mean if upd else None), ptr(running_var if upd else None), ptr(pro), ptr(sums), M,
                      C, float(eps), float(momentum), stream_ptr(dev))
        wk = _weight_layout(weight, C, "krsc")
        P, Q = _out_hw(H, W, R, S, stride, pad)
        out = torch.empty((N, Cout, P, Q), dtype=y.dtype, device=dev, memory_format=torch.channels_last)
        st = None
        if want_stats:
            st = torch.empty(2 * Cout, dtype=torch.float32, device=dev)
        ws = _conv_ws(N * P * Q, Cout, R * S * C, False, dev)
        if want_stats and bnfin is not None:
            _conv_fwd_bn(bnfin, ys, wk, out, st, ws, (N, H, W, C, P, Q, Cout, R, S, stride, pad), pro, dev)
        else:
            _lib.call("tdl_conv_nt_pro", ptr(ys), ptr(wk), ptr(out), ptr(st), ptr(ws), N, H, W, C, P, Q, Cout, R, S,
                      stride, pad, ptr(pro), stream_ptr(dev))
        ctx.save_for_backward(ys, bnp, gamma, weight)
        ctx.sums = sums
        ctx.beta = beta  # a parameter (leaf): only its identity / main_grad is needed
        ctx.geom = (N, C, H, W, Cout, R, S, P, Q, stride, pad)
        ctx.set_materialize_grads(False)   # no zero-filled gradient for the statistics output
        if st is None:
            st = torch.zeros(0, dtype=torch.float32, device=dev)
        ctx.mark_non_differentiable(st)
        return out, st

    @staticmethod
    def backward(ctx, dout, _dstats):
        if dout is None:
            return (None,) * 14
        ys, bnp, gamma, weight = ctx.saved_tensors
        C_ = ys.shape[1]
        pro, mean, rstd = bnp[:2 * C_], bnp[2 * C_:3 * C_], bnp[3 * C_:]
        N, C, H, W, Cout, R, S, P, Q, stride, pad = ctx.geom
        dev = dout.device
        dout = dout.contiguous(memory_format=torch.channels_last)
        if dout.dtype != ys.dtype:
            dout = dout.to(ys.dtype)
        # data gradient of the conv = gradient w.r.t. the (never stored) BN output; its epilogue also
        # reduces the BN backward's per-channel sums (ReLU mask recomputed from y), so the BN
        # backward below is the elementwise pass only
        # (the completed sums are also the BN's bias / scale gradients: added into dbeta / dgamma there)
        beta = ctx.beta
        mg_g, mg_b = getattr(gamma, "main_grad", None), getattr(beta, "main_grad", None)
        dg = mg_g if mg_g is not None else torch.zeros(C, dtype=torch.float32, device=dev)
        db = mg_b if mg_b is not None else torch.zeros(C, dtype=torch.float32, device=dev)
        wd = _weight_layout(weight, C, "crsk")  # [C][R][S][Cout]
        dbn = torch.empty((N, C, H, W), dtype=dout.dtype, device=dev, memory_format=torch.channels_last)
        ws = _conv_ws(N * H * W, C, R * S * Cout, stride == 2, dev)
        _lib.call("tdl_conv_dgrad_bnsums", ptr(dout), ptr(wd), ptr(dbn), ptr(ws), N, P, Q, Cout, H, W, C, R, S, stride,
                  pad, ptr(ys), ptr(bnp), ptr(ctx.sums), ptr(dg), ptr(db), stream_ptr(dev))
        # weight gradient against relu(BN(y)) recomputed on load
        gw = None
        if ctx.needs_input_grad[8]:
            mg = getattr(weight, "main_grad", None)
            acc = mg if (mg is not None and mg.is_contiguous()) else torch.zeros((Cout, C, R, S), dtype=torch.float32,
                                                                                 device=dev)
            wsw = torch.empty(Cout * R * S * C, dtype=torch.float32, device=dev) if R * S > 1 else None

            def _wg():
                _lib.call("tdl_conv_wgrad_pro", ptr(dout), ptr(ys), ptr(acc), ptr(wsw), N, H, W, C, P, Q, Cout, R, S,
                          stride, pad, _num_cu(dev), ptr(pro), stream_ptr(dev))
            if acc is mg:
                _wgrad(dev, _wg, (dout, ys, wsw, bnp))
            else:
                _wg()
            if acc is not mg:
                if mg is not None:
                    mg.add_(acc)
                else:
                    gw = acc.to(weight.dtype)
        # BN (+ ReLU) backward with the mask recomputed from y
        dy = torch.empty_like(ys, memory_format=torch.channels_last)
        _lib.call("tdl_bn_act_bwd_pro_summed", ptr(dbn), ptr(ys), ptr(mean), ptr(rstd), ptr(gamma), ptr(pro),
                  ptr(ctx.sums), ptr(dy), N * H * W, C, stream_ptr(dev))
        gg = None if mg_g is not None else dg.to(gamma.dtype)
        gb = None if mg_b is not None else db.to(beta.dtype)
        return dy, None, gg, gb, None, None, None, None, gw, None, None, None, None, None


def _bn_fold_enabled() -> bool:
    return os.environ.get("TDL_BN_FOLD", "1") != "0"


def conv_bn_chain(x: torch.Tensor, units, relu: bool = True, residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``units`` = [(conv, bn), ...]: relu(bn(conv(...relu(bn(conv(x)))...)) (+ residual)) with ReLU after
    every intermediate BN.  On the native training path each intermediate BN + ReLU is folded into
    the next convolution (``_BNActConvNHWC``: its output is never written); otherwise the units run
    one by one through ``conv_bn_act``."""
    units = list(units)
    if not (native_conv_ok(x) and _bn_fold_enabled() and all(bn.training for _, bn in units)) or len(units) == 1:
        for i, (conv, bn) in enumerate(units):
            last = i == len(units) - 1
            x = conv_bn_act(x, conv, bn, relu=relu if last else True, residual=residual if last else None)
        return x
    conv0, _ = units[0]
    if conv0.bias is not None:
        raise NotImplementedError("native conv: bias")
    # each folded BN is finalized by the kernels of the convolution producing its input
    fins = [{"bn": bn} for _, bn in units[:-1]] + [None]
    y, stats = _Conv2dNHWC.apply(x, conv0.weight, _single(conv0.stride), _single(conv0.padding), True, fins[0])
    for i, ((_, bn), (conv, _)) in enumerate(zip(units[:-1], units[1:])):
        if conv.groups != 1 or _single(conv.dilation) != 1 or conv.bias is not None \
                or conv.kernel_size[0] != conv.kernel_size[1]:
            raise NotImplementedError(f"native conv: unsupported configuration {conv}")
        momentum = bn.momentum if bn.momentum is not None else 0.1
        y, stats = _BNActConvNHWC.apply(y, stats, bn.weight, bn.bias, bn.running_mean, bn.running_var, momentum, bn.eps,
                                        conv.weight, _single(conv.stride), _single(conv.padding), True, fins[i],
                                        fins[i + 1])
    bn = units[-1][1]
    momentum = bn.momentum if bn.momentum is not None else 0.1
    return _BatchNormActNHWC.apply(y, stats, bn.weight, bn.bias, residual, bn.running_mean, bn.running_var, True,
                                   momentum, bn.eps, relu)


class _MaxPoolNHWC(torch.autograd.Function):
    """Max-pool on NHWC bf16 (csrc/pool.hip): the window argmax is kept as one byte per output
    element and the backward gathers (deterministic, no atomics)."""

    @staticmethod
    def forward(ctx, x, k: int, stride: int, pad: int):
        N, C, H, W = x.shape
        xs = x.contiguous(memory_format=torch.channels_last)
        P, Q = _out_hw(H, W, k, k, stride, pad)
        y = torch.empty((N, C, P, Q), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        arg = torch.empty((N, P, Q, C), dtype=torch.uint8, device=x.device)
        _lib.call("tdl_maxpool_fwd", ptr(xs), ptr(y), ptr(arg), N, H, W, C, P, Q, k, k, stride, pad,
                  stream_ptr(x.device))
        ctx.save_for_backward(arg)
        ctx.geom = (N, C, H, W, P, Q, k, stride, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        N, C, H, W, P, Q, k, stride, pad = ctx.geom
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = torch.empty((N, C, H, W), dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
        _lib.call("tdl_maxpool_bwd", ptr(dy), ptr(arg), ptr(dx), N, H, W, C, P, Q, k, k, stride, pad,
                  stream_ptr(dy.device))
        return dx, None, None, None


class _GlobalAvgPoolNHWC(torch.autograd.Function):
    """[N, C, H, W] (channels_last bf16) -> [N, C] mean over H*W (csrc/pool.hip)."""

    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        xs = x.contiguous(memory_format=torch.channels_last)
        y = torch.empty((N, C), dtype=x.dtype, device=x.device)
        _lib.call("tdl_global_avgpool_fwd", ptr(xs), ptr(y), N, H * W, C, stream_ptr(x.device))
        ctx.shape = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        N, C, H, W = ctx.shape
        dy = dy.contiguous()
        dx = torch.empty((N, C, H, W), dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
        _lib.call("tdl_global_avgpool_bwd", ptr(dy), ptr(dx), N, H * W, C, stream_ptr(dy.device))
        return dx


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """``F.adaptive_avg_pool2d(x, 1).flatten(1)``; native NHWC kernels for CUDA bf16 with C % 8 == 0."""
    if native_conv_ok(x) and x.shape[1] % 8 == 0:
        return _GlobalAvgPoolNHWC.apply(x)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


def max_pool2d(x: torch.Tensor, kernel_size: int, stride: Optional[int] = None, padding: int = 0) -> torch.Tensor:
    """``F.max_pool2d`` (square window, floor mode); native NHWC kernels for CUDA bf16 with C % 8 == 0."""
    stride = kernel_size if stride is None else stride
    if native_conv_ok(x) and x.shape[1] % 8 == 0:
        return _MaxPoolNHWC.apply(x, int(kernel_size), int(stride), int(padding))
    return F.max_pool2d(x, kernel_size, stride, padding)


def _single(v) -> int:
    return int(v if isinstance(v, int) else v[0])


def conv_bn_act(x: torch.Tensor, conv: nn.Conv2d, bn: nn.BatchNorm2d, relu: bool = True,
                residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """act(bn(conv(x)) (+ residual)).  Native NHWC kernels for CUDA bf16, the torch modules otherwise."""
    if not native_conv_ok(x):
        out = bn(conv(x))
        if residual is not None:
            out = out + residual
        return F.relu(out) if relu else out
    if conv.groups != 1 or _single(conv.dilation) != 1 or conv.bias is not None \
            or conv.kernel_size[0] != conv.kernel_size[1] or conv.stride[0] != conv.stride[-1] \
            or conv.padding[0] != conv.padding[-1]:
        raise NotImplementedError(f"native conv: unsupported configuration {conv}")
    training = bn.training
    y, stats = _Conv2dNHWC.apply(x, conv.weight, _single(conv.stride), _single(conv.padding), training)
    momentum = bn.momentum if bn.momentum is not None else 0.1
    return _BatchNormActNHWC.apply(y, stats, bn.weight, bn.bias, residual, bn.running_mean, bn.running_var,
                                   training, momentum, bn.eps, relu)


def conv2d(x: torch.Tensor, weight: torch.Tensor, stride: int = 1, padding: int = 0) -> torch.Tensor:
    """Plain convolution (no BN) on the native path for CUDA bf16 tensors."""
    if native_conv_ok(x):
        y, _ = _Conv2dNHWC.apply(x, weight, int(stride), int(padding), False)
        return y
    return F.conv2d(x, weight, None, stride, padding)
