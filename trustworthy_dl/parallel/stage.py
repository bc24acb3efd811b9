"""One pipeline stage: its layer modules, flat parameter buffers and device verifier.

A stage owns a contiguous range ``[a, b)`` of the model's ``pipeline_layers()``.  Its module is
an ``nn.Sequential`` of (deep copies of) those layers, so stage-local parameter names are
``"<i>.<name>"`` exactly like the reference's ``nn.Sequential(h[i:j])`` partitions
(distributed_trainer.py:132-134; checkpoint layout 448-459).
"""
from __future__ import annotations

import copy
import functools
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from .flat import FlatParams
from ..security.stage_verifier import StageVerifier


def tied_groups(model: nn.Module) -> List[List[Tuple[int, str]]]:
    """Parameters shared between pipeline layers, as lists of (layer index, attribute)."""
    layers = model.pipeline_layers()
    by_id: Dict[int, List[Tuple[int, str]]] = {}
    for li, layer in enumerate(layers):
        for name, p in layer.named_parameters(recurse=False):
            by_id.setdefault(id(p), []).append((li, name))
        for mname, m in layer.named_modules():
            if not mname:
                continue
            for pname, p in m.named_parameters(recurse=False):
                by_id.setdefault(id(p), []).append((li, f"{mname}.{pname}"))
    return [v for v in by_id.values() if len({li for li, _ in v}) > 1]


class Stage:
    def __init__(self, model: nn.Module, layer_range: Tuple[int, int], stage_id: int, num_stages: int,
                 device, compute_dtype: torch.dtype, verifier_kwargs: Optional[dict] = None,
                 layers: Optional[List[nn.Module]] = None):
        self.layer_range = tuple(layer_range)
        self.stage_id = stage_id
        self.num_stages = num_stages
        self.device = torch.device(device)
        self.compute_dtype = compute_dtype
        a, b = self.layer_range
        if layers is None:
            layers = copy.deepcopy(model.pipeline_layers()[a:b])
        # fp32 on the device first: FlatParams copies the fp32 init into the master buffer and
        # then re-binds every parameter to its compute-dtype (bf16) view
        self.module = nn.Sequential(*layers).to(self.device)
        self.takes_tokens = bool(getattr(layers[0], "takes_tokens", False)) or a == 0
        self.computes_loss = bool(getattr(layers[-1], "computes_loss", False))
        self.flat = FlatParams(self.module, self.device, compute_dtype)
        self._hooks = []
        for p in self.flat.params:
            self._hooks.append(p.register_post_accumulate_grad_hook(self._fold_grad))
        vk = dict(verifier_kwargs or {})
        self.verifier = StageVerifier(self.flat.sizes, self.device, **vk)
        self.clip_excluded: List[Tuple[int, int]] = []
        # weight-integrity checksums (parallel/attribution.py): post-update commitment, the checksum
        # of the weights in use this step, one taken early on the side stream, the tail re-check
        self.param_checksum: Optional[torch.Tensor] = None
        self._cur_checksum: Optional[torch.Tensor] = None
        self._early_checksum: Optional[torch.Tensor] = None
        self._tail_flag: Optional[torch.Tensor] = None

    def set_clip_exclusions(self, excluded_ids) -> None:
        """Parameters whose gradient another stage already counts in the global clipping norm (the
        non-owner copies of a tied weight, e.g. the LM head's ``wte`` on the last stage: after the
        tied all-reduce both copies hold the same summed gradient).  A single optimizer over the
        whole model (reference distributed_trainer.py:441-446) sees that gradient once."""
        ex = set(excluded_ids)
        self.clip_excluded = [(o, n) for q, o, n in zip(self.flat.params, self.flat.offsets, self.flat.sizes)
                              if id(q) in ex]
        self.verifier.set_clip_weights([0.0 if id(q) in ex else 1.0 for q in self.flat.params])

    def clip_sumsq(self, grad: torch.Tensor) -> torch.Tensor:
        """Sum of squares of ``grad`` (this stage's flat gradient) over the parameters this stage
        counts for clipping (device scalar)."""
        from ..security.grad_audit import _segments, seg_sumsq
        return seg_sumsq(grad, _segments(grad.numel(), [(o, o + n) for o, n in self.clip_excluded]))

    @staticmethod
    def _fold_grad(p: torch.Tensor):
        """Modules not routed through the fused ops (convs, BN, nn.Linear) produce ``.grad``;
        fold it into the flat fp32 accumulator so every stage verifies/steps one buffer."""
        if p.grad is not None:
            p.main_grad.add_(p.grad.float())
            p.grad = None

    @property
    def is_first(self) -> bool:
        return self.layer_range[0] == 0

    def _runners(self) -> List:
        """Callables over the stage's layers: an adjacent (attn, mlp) half-block pair of the same
        block runs as one fused block (models/gpt2.py FusedHalfPair)."""
        r = getattr(self, "_runner_cache", None)
        if r is not None:
            return r
        from ..models.gpt2 import FusedHalfPair, GPT2HalfBlock
        layers, out, i = list(self.module), [], 0
        self._runner_layer_idx: List[List[int]] = []
        while i < len(layers):
            a = layers[i]
            b = layers[i + 1] if i + 1 < len(layers) else None
            if (isinstance(a, GPT2HalfBlock) and isinstance(b, GPT2HalfBlock) and a.part == "attn"
                    and b.part == "mlp" and a.block_index == b.block_index):
                out.append(FusedHalfPair(a, b))
                self._runner_layer_idx.append([i, i + 1])
                i += 2
            else:
                out.append(a)
                self._runner_layer_idx.append([i])
                i += 1
        self._runner_cache = out
        return out

    # ---------------------------------------------------------------- verification overlap
    def set_early_stats(self, excluded_ids=()) -> None:
        """Prepare the per-layer gradient-statistics triggers: for each stage-local layer, the runs
        of flat segments (parameters) it owns.  Parameters in ``excluded_ids`` (tied weights, whose
        gradient changes in the tied all-reduce after the backward) are left to the final pass."""
        ex = set(excluded_ids)
        per_layer: Dict[int, List[int]] = {}
        self._tied_layers = set()
        for j, (name, q) in enumerate(zip(self.flat.names, self.flat.params)):
            if id(q) in ex:
                self._tied_layers.add(int(name.split(".", 1)[0]))
                continue
            per_layer.setdefault(int(name.split(".", 1)[0]), []).append(j)
        self._layer_seg_runs = {}
        for li, segs in per_layer.items():
            runs, lo = [], segs[0]
            for a, b in zip(segs, segs[1:] + [None]):
                if b != a + 1:
                    runs.append((lo, a + 1))
                    lo = b
            self._layer_seg_runs[li] = runs

    def _fused_mode(self) -> str:
        """Where the last micro-batch's split-K weight-gradient reduce runs (TDL_FUSED_GRAD_STATS):
        "side" — fused with the verifier's statistics (ops/stats.py reduce_partial) on the
        verifier's side stream, so the compute stream carries neither (only where nothing reads
        the gradient before the step tail: ``side_reduce_ok``, set by the engine; measured 0.4 %
        slower than "0": the reduce traffic then competes with the backward's GEMMs,
        profiles/r6_side_reduce_ab.txt); "1" — fused, on the compute stream (1.4 % slower:
        profiles/r3_fused_grad_stats_ab.txt); "0" (default) — a reduce pass on the compute stream
        and the statistics on the side stream."""
        m = os.environ.get("TDL_FUSED_GRAD_STATS", "0")
        if m == "auto":
            m = "side" if getattr(self, "side_reduce_ok", False) and self.verifier.side is not None else "0"
        return m

    def _arm_sinks(self, runner_idx: int):
        """Autograd hook body: runner ``runner_idx`` is about to run its backward for the step's
        last micro-batch -> arm the verifier's fused split-K reduce on its (untied) weight
        gradients: that backward's weight-gradient GEMM then hands its fp32 slabs to one kernel
        that completes each gradient and takes its statistics (ops/stats.py reduce_partial),
        instead of a reduce pass plus a side-stream pass re-reading the final gradient."""
        gs = self.verifier.grad_stats
        mode = self._fused_mode()
        if gs is None or not self.verifier.verify_on or mode == "0":
            return
        sink = self._fused_sink_side if mode == "side" else self._fused_sink
        for li in self._runner_layer_idx[runner_idx]:
            for lo, hi in self._layer_seg_runs.get(li, []):
                for j in range(lo, hi):
                    mg = getattr(self.flat.params[j], "main_grad", None)
                    if mg is not None and mg.dim() == 2:
                        mg._tdl_stats_sink = functools.partial(sink, j)

    def _fused_sink(self, seg: int, slabs, nsplit: int) -> bool:
        return self.verifier.grad_stats.reduce_partial(self.flat.grad, seg, slabs, nsplit)

    def _fused_sink_side(self, seg: int, slabs, nsplit: int) -> bool:
        """The fused reduce on the verifier's side stream, ordered after the GEMM that wrote the
        slabs; the slabs stay allocated until it ran; ``finish_step`` joins the stream before
        anything reads the gradient."""
        side = self.verifier.side
        side.wait_stream(torch.cuda.current_stream(slabs.device))
        with torch.cuda.stream(side):
            ok = self.verifier.grad_stats.reduce_partial(self.flat.grad, seg, slabs, nsplit)
        slabs.record_stream(side)
        return ok

    def _grad_ready(self, runner_idx: int):
        """Autograd hook body: runner ``runner_idx``'s backward (incl. weight gradients) of the
        step's last micro-batch is done -> its layers' gradient statistics can start (segments
        already covered by a fused reduce are skipped)."""
        runs = []
        gs = self.verifier.grad_stats
        fused = gs.fused_segs if gs is not None else ()
        for li in self._runner_layer_idx[runner_idx]:
            for lo, hi in self._layer_seg_runs.get(li, []):
                j = lo
                while j < hi:
                    if j in fused:
                        j += 1
                        continue
                    k = j
                    while k < hi and k not in fused:
                        k += 1
                    runs.append((j, k))
                    j = k
        if runs:
            self.verifier.grad_ready(self.flat.grad, runs)
        cb = getattr(self, "on_tied_ready", None)
        if cb is not None and any(li in getattr(self, "_tied_layers", ()) for li in self._runner_layer_idx[runner_idx]):
            cb()  # a tied weight's gradient is final: its cross-stage all-reduce can start

    def forward(self, x, labels=None, observe=None, arm_grad_stats: bool = False):
        """Returns (output, monitored_activation).  Loss stages return the (scalar) loss.

        ``observe``: optional output monitor.  A loss layer that owns its monitored tensor (the
        fused LM head: logits are rewritten into dlogits in place) is handed it and calls it at the
        right moment; the returned monitored activation is then None (already observed).

        ``arm_grad_stats`` (the step's last micro-batch, weight gradients not deferred): hook every
        layer input so that layer's gradient statistics start on the verifier's side stream as
        soon as its backward is done, overlapping the backward of the layers before it."""
        layers = self._runners()
        if x.is_cuda:
            cw = getattr(self, "_conv_weights", None)
            if cw is None:   # the stage's conv weights (bf16 views into the flat buffer)
                cw = self._conv_weights = [m.weight for m in self.module.modules() if isinstance(m, nn.Conv2d)]
            if cw:   # their kernel layouts for this weight generation, batched (ops/conv.py)
                from ..ops.conv import prebuild_layouts
                prebuild_layouts(cw)
            mw = getattr(self, "_matrix_weights", None)
            if mw is None:   # 2-D weights: their forward-layout copies, batched (ops/layers.py)
                mw = self._matrix_weights = [p for p in self.module.parameters() if p.dim() == 2]
            if mw and os.environ.get("TDL_FWD_PREBUILD", "1") != "0":   # (A/B switch)
                from ..ops.layers import prebuild_fwd_weights
                prebuild_fwd_weights(mw)
        arm = arm_grad_stats and getattr(self, "_layer_seg_runs", None) is not None
        for k, layer in enumerate(layers[:-1]):
            if arm and x.requires_grad:
                x.register_hook(lambda g, k=k: self._grad_ready(k))
            x = layer(x)
            if arm and x.requires_grad:   # fires right before runner k's backward
                x.register_hook(lambda g, k=k: self._arm_sinks(k))
        last = layers[-1]
        if arm and x.requires_grad:
            x.register_hook(lambda g, k=len(layers) - 1: self._grad_ready(k))
        out = self._forward_last(last, x, labels, observe)
        if arm:
            y = out[0]
            if isinstance(y, torch.Tensor) and y.requires_grad:
                y.register_hook(lambda g, k=len(layers) - 1: self._arm_sinks(k))
        return out

    def _forward_last(self, last, x, labels, observe):
        layers = self._runners()
        if self.computes_loss:
            mon = x if len(layers) > 1 else None
            if mon is None and observe is not None and getattr(last, "accepts_observer", False):
                last._observe = observe
                try:
                    out = last(x, labels)
                finally:
                    last._observe = None
                return out, None
            out = last(x, labels)
            if mon is None:
                mon = getattr(last, "_last_logits", None)
            return out, mon
        y = last(x)
        return y, y

    def output_observer(self):
        """Monitor callable for this stage's output: queue its statistics on the verifier's side
        stream, then make the compute stream wait for them (the tensor may be overwritten next)."""
        def observe(t: torch.Tensor):
            self.verifier.observe_output(t)
            if self.verifier.side is not None:
                torch.cuda.current_stream(self.device).wait_stream(self.verifier.side)
        return observe

    def local_param(self, layer_idx: int, attr: str) -> Optional[nn.Parameter]:
        a, b = self.layer_range
        if not a <= layer_idx < b:
            return None
        mod = self.module[layer_idx - a]
        obj = mod
        for part in attr.split("."):
            obj = getattr(obj, part)
        return obj

    # ---------------------------------------------------------------- migration helpers
    def layer_state(self, layer_idx: int) -> Dict[str, torch.Tensor]:
        """fp32 master / exp_avg / exp_avg_sq of one layer's parameters, keyed by layer-local name."""
        a, _ = self.layer_range
        pre = f"{layer_idx - a}."
        out = {}
        for i, n in enumerate(self.flat.names):
            if n.startswith(pre):
                local = n[len(pre):]
                out[local] = torch.stack([self.flat.view(self.flat.master, i).reshape(-1),
                                          self.flat.view(self.flat.exp_avg, i).reshape(-1),
                                          self.flat.view(self.flat.exp_avg_sq, i).reshape(-1)])
        return out

    def buffers_state(self) -> Dict[str, torch.Tensor]:
        return {k: v.detach().clone() for k, v in self.module.named_buffers()}

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
