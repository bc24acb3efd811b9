"""Flat parameter / gradient / optimizer-state buffers for one pipeline stage.

Every stage re-homes its parameters into contiguous buffers:

* ``data``      model-visible weights (bf16 on GPU, fp32 on CPU); each ``nn.Parameter`` is a view
* ``master``    fp32 master weights (aliases ``data`` when the compute dtype is fp32)
* ``exp_avg``, ``exp_avg_sq``  AdamW moments, fp32
* ``grad``      fp32 gradient accumulator; every parameter gets ``.main_grad`` = its view

so that (a) the fused AdamW is one bandwidth-bound launch per weight-decay group
(csrc/optim.hip), (b) gradient verification is one segmented reduction over ``grad``
(csrc/stats.hip K3), and (c) re-sharding a stage to another GPU is a handful of large
contiguous P2P transfers over xGMI (``PipelineEngine._migrate`` in parallel/pipeline.py) instead
of hundreds of small ones.
Parameters are ordered [weight-decay group | no-decay group] (biases, LayerNorm, embeddings
of positions are not decayed).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from ..ops import _lib
from ..ops._lib import ptr, stream_ptr
from ..ops.layers import bump_weight_generation


def _no_decay(name: str, p: torch.Tensor) -> bool:
    return p.ndim < 2 or "ln" in name or "norm" in name or "bn" in name or name.endswith("bias") \
        or "wpe" in name


@dataclass
class AdamWConfig:
    lr: float = 5e-5
    betas: Tuple[float, float] = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.01
    max_grad_norm: float = 0.0  # 0 disables clipping
    warmup_steps: int = 0       # linear learning-rate warm-up over this many optimizer steps

    def lr_at(self, step: int) -> float:
        if self.warmup_steps > 0 and step < self.warmup_steps:
            return self.lr * step / self.warmup_steps
        return self.lr


class FlatParams:
    def __init__(self, module: nn.Module, device, compute_dtype: torch.dtype = torch.float32,
                 shared: Optional[Dict[str, str]] = None):
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        named = []
        seen = set()
        for name, p in module.named_parameters():
            if id(p) in seen:
                continue
            seen.add(id(p))
            named.append((name, p))
        named.sort(key=lambda np_: _no_decay(*np_))  # stable: decay group first
        self.names = [n for n, _ in named]
        self.params = [p for _, p in named]
        self.sizes = [p.numel() for p in self.params]
        self.shapes = [tuple(p.shape) for p in self.params]
        self.offsets = [0]
        for s in self.sizes:
            self.offsets.append(self.offsets[-1] + s)
        self.numel = self.offsets[-1]
        self.n_decay = sum(1 for n, p in named if not _no_decay(n, p))
        self.decay_numel = self.offsets[self.n_decay]

        self.master = torch.empty(self.numel, dtype=torch.float32, device=self.device)
        for p, o, s in zip(self.params, self.offsets, self.sizes):
            self.master[o:o + s].copy_(p.detach().reshape(-1).float())
        if compute_dtype == torch.float32:
            self.data = self.master
        else:
            self.data = self.master.to(compute_dtype)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.exp_avg = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.exp_avg_sq = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
        self.step_count = 0
        self._rebind()

    def _rebind(self):
        """Point every parameter at its slice of ``data`` and attach ``.main_grad``."""
        for p, o, s, shp in zip(self.params, self.offsets, self.sizes, self.shapes):
            p.data = self.data[o:o + s].view(shp)
            p.main_grad = self.grad[o:o + s].view(shp)
            p.grad = None

    def set_grad_buffer(self, buf: torch.Tensor) -> torch.Tensor:
        """Re-point every parameter's ``main_grad`` at ``buf`` (same layout as ``grad``) and return
        the previous accumulator: the backward audit recomputes one micro-batch's gradient into a
        scratch buffer without touching the step's accumulated gradient."""
        old = self.grad
        self.grad = buf
        for p, o, s, shp in zip(self.params, self.offsets, self.sizes, self.shapes):
            p.main_grad = buf[o:o + s].view(shp)
        return old

    def view(self, buf: torch.Tensor, i: int) -> torch.Tensor:
        return buf[self.offsets[i]:self.offsets[i + 1]].view(self.shapes[i])

    # ------------------------------------------------------------------ optimizer
    def zero_grad(self):
        self.grad.zero_()

    def adamw_step(self, cfg: AdamWConfig, ctrl: Optional[torch.Tensor] = None, zero_grad: bool = True):
        """Fused AdamW on both weight-decay groups.  ``ctrl`` (device f32[2]) = (grad scale, skip)."""
        self.step_count += 1
        t = self.step_count
        b1, b2 = cfg.betas
        bc1, bc2 = 1.0 - b1 ** t, 1.0 - b2 ** t
        lr = cfg.lr_at(t)
        groups = [(0, self.decay_numel, cfg.weight_decay), (self.decay_numel, self.numel, 0.0)]
        if self.device.type == "cuda":
            for lo, hi, wd in groups:
                n = hi - lo
                if n <= 0:
                    continue
                _lib.call("tdl_adamw_flat", ptr(self.master[lo:]), ptr(self.exp_avg[lo:]), ptr(self.exp_avg_sq[lo:]),
                          ptr(self.grad[lo:]), ptr(None if self.data is self.master else self.data[lo:]),
                          n, lr, b1, b2, cfg.eps, wd, bc1, bc2,
                          ptr(ctrl), int(zero_grad), stream_ptr(self.device))
            bump_weight_generation()   # compute weights rewritten in place: forward-layout copies are stale
            return
        scale = 1.0 if ctrl is None else float(ctrl[0])
        skip = False if ctrl is None else bool(float(ctrl[1]) != 0.0)
        if not skip:
            for lo, hi, wd in groups:
                if hi <= lo:
                    continue
                g = self.grad[lo:hi] * scale
                m, v, p = self.exp_avg[lo:hi], self.exp_avg_sq[lo:hi], self.master[lo:hi]
                m.mul_(b1).add_(g, alpha=1 - b1)
                v.mul_(b2).addcmul_(g, g, value=1 - b2)
                p.mul_(1 - lr * wd)
                p.addcdiv_(m, (v.sqrt() / math.sqrt(bc2)).add_(cfg.eps), value=-lr / bc1)
            if self.data is not self.master:
                self.data.copy_(self.master)
        if zero_grad:
            self.grad.zero_()

    # ------------------------------------------------------------------ state
    def state_dict(self) -> Dict:
        return {"names": list(self.names), "shapes": list(self.shapes), "step": self.step_count,
                "master": self.master.detach().cpu(), "exp_avg": self.exp_avg.detach().cpu(),
                "exp_avg_sq": self.exp_avg_sq.detach().cpu()}

    def load_state_dict(self, sd: Dict):
        if list(sd["names"]) != self.names:
            # tolerate reordering: map by name
            src = {n: i for i, n in enumerate(sd["names"])}
            offs = [0]
            for shp in sd["shapes"]:
                offs.append(offs[-1] + int(torch.Size(shp).numel()))
            for i, n in enumerate(self.names):
                j = src[n]
                for key, dst in (("master", self.master), ("exp_avg", self.exp_avg), ("exp_avg_sq", self.exp_avg_sq)):
                    dst[self.offsets[i]:self.offsets[i + 1]].copy_(sd[key][offs[j]:offs[j + 1]])
        else:
            self.master.copy_(sd["master"])
            self.exp_avg.copy_(sd["exp_avg"])
            self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.step_count = int(sd["step"])
        if self.data is not self.master:
            self.data.copy_(self.master)

    def optimizer_state_tensors(self) -> List[torch.Tensor]:
        return [self.master, self.exp_avg, self.exp_avg_sq]
