"""Device-resident verification of one pipeline stage (the engine's fast path).

Per training step, without any host synchronisation:

1. output statistics of the stage's first micro-batch output (K1+K2, on a side HIP stream so it
   overlaps the next micro-batch's compute) -> z-score decision against a device ring baseline (K4);
2. segmented gradient statistics over the stage's flat fp32 gradient (K3: per-parameter norms,
   cosine vs an EMA reference gradient, moments, quantiles, non-finite count) -> z-score decision;
3. trust metrics (reference formulas distributed_trainer.py:228-271, with the symmetric
   gradient-consistency fix) from device EMA baselines;
4. a fixed-size float "digest" row that the engine all-gathers across ranks; every rank then
   runs the fused trust update (K5) on identical data, and the optimizer reads a 2-float control
   block (grad scale, skip) written here — a flagged gradient is quarantined on device.

The host mirrors (TrustManager / AttackDetector / attack_history) are fed from the digests one
step later through a pinned, non-blocking copy.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

import torch

from ..ops import stats as S

# TDL_VERIFY_FUSED=0: the torch form of the step tail on the GPU too (A/B and cross-check)
VERIFY_FUSED = os.environ.get("TDL_VERIFY_FUSED", "1") != "0"


class _FinishArgs(ctypes.Structure):
    """csrc/stats.hip VerifyFinishArgs (field order and types must match)."""
    _fields_ = [("d", ctypes.c_void_p), ("loss", ctypes.c_void_p), ("stage_id", ctypes.c_int),
                ("out_on", ctypes.c_int), ("out_res", ctypes.c_void_p), ("out_stats", ctypes.c_void_p),
                ("out_mu", ctypes.c_void_p), ("out_sd", ctypes.c_void_p), ("out_n", ctypes.c_void_p),
                ("warmup", ctypes.c_float), ("deadzone", ctypes.c_float), ("beta", ctypes.c_float),
                ("grad_mode", ctypes.c_int), ("sumsq_bare", ctypes.c_void_p), ("g", ctypes.c_void_p),
                ("S", ctypes.c_int), ("clip_w", ctypes.c_void_p), ("gdet", ctypes.c_int),
                ("grad_res", ctypes.c_void_p), ("targeted", ctypes.c_int), ("sign_flip_cos", ctypes.c_float),
                ("norm_ema", ctypes.c_void_p), ("norm_n", ctypes.c_void_p), ("tol", ctypes.c_float),
                ("symmetric", ctypes.c_int), ("hm0", ctypes.c_float), ("hm1", ctypes.c_float),
                ("hm2", ctypes.c_float), ("hm3", ctypes.c_float), ("truth", ctypes.c_int),
                ("quarantine", ctypes.c_int), ("ctrl", ctypes.c_void_p)]

# digest layout (floats)
D_LOSS, D_OUT_FLAG, D_OUT_Z, D_GRAD_FLAG, D_GRAD_Z = 0, 1, 2, 3, 4
D_METRICS = 5  # 6 trust metrics: output_deviation, gradient_consistency, latency, utilization, error, uptime
D_GRAD_SUMSQ, D_OUT_MEAN, D_OUT_STD, D_GRAD_L2, D_NONFINITE, D_GRAD_COS = 11, 12, 13, 14, 15, 16
D_ATTACK_TRUTH, D_PRESENT, D_STAGE, D_OUT_CONF, D_GRAD_CONF = 17, 18, 19, 20, 21
D_OFFLINE_MASK = 22  # bitmask of the peers this rank's heartbeat watchdog sees offline
D_PARAM_FLAG = 23    # compute weights changed outside the optimizer (integrity checksum mismatch)
D_AUDIT_PREV = 24    # recompute audit of the PREVIOUS stage's monitored micro-batch: 1 = its output did
                     # not match f(input; weights) recomputed here (parallel/pipeline.py _audit)
D_AUDITED_PREV = 25  # 1 when that audit ran this step
D_AUDIT_ERR = 26     # its relative max error
# backward audit (parallel/audit.py, parallel/commitments.py, security/grad_audit.py)
D_AUDIT_KIND_PREV = 27  # bitmask of the failed checks behind D_AUDIT_PREV (AK_* below)
D_AUDIT_NEXT = 28    # audit of the NEXT stage when it is the loss stage (its predecessor audits it)
D_AUDITED_NEXT = 29
D_AUDIT_KIND_NEXT = 30
# 31-35 unused (r5's self-reported tied-weight sketches)
D_MIRROR = 36        # 1 when this rank checked its audited stages against live optimizer mirrors this step
# cross-party hashes: the first 128 bits of BLAKE2s Merkle roots as 8 exact 16-bit halves each
# (grad_audit.hash_row); -1 = none this step
D_WHASH = 37         # [8] (weight-shipping mode) root of this stage's compute weights after its last update
D_WHASH_PREV = 45    # [8] root of the weights the audited previous stage shipped here
D_WHASH_NEXT = 53    # [8] same for the audited next (loss) stage
D_DXHASH_RECV = 61   # [8] root of the input gradients received from the next stage for the micro-batches
                     #     that stage's auditor opened (distributed)
D_DXHASH_SHIP = 69   # [8] root of the input gradients the audited previous stage shipped here
D_XHASH_SENT = 77    # [8] root of the outputs this stage SENT to the next stage for the micro-batches
                     #     that stage's auditor opened (= their inputs)
D_XHASH_SHIP = 85    # [8] root of the inputs the audited previous stage shipped here
D_SUMSQ_PREV = 93    # (mirror mode) clipping sum of squares of the gradient the audited previous stage
                     #     shipped here, computed by this auditor (-1: none); the global clip uses these
D_SUMSQ_NEXT = 94    # same for the audited next (loss) stage
# tied weight (mirror mode): for an audited previous / next stage holding a member of the tie group,
# computed by this auditor under the step's shared tie key: U = sum of its M committed tied
# contribution sketches (each opened one verified), G = sketch of the tied gradient it shipped and
# applies, N = that gradient's norm, ON = 1 when set (parallel/commitments.py ``_tied_mismatch``)
D_TIE_U_PREV, D_TIE_G_PREV, D_TIE_N_PREV, D_TIE_ON_PREV = 95, 99, 103, 104
D_TIE_U_NEXT, D_TIE_G_NEXT, D_TIE_N_NEXT, D_TIE_ON_NEXT = 105, 109, 113, 114
DIGEST = 115         # csrc/stats.hip VD_DIGEST
# audit check bits
AK_FWD, AK_DX, AK_DW, AK_WHASH, AK_DXHASH, AK_GAPP = 1, 2, 4, 8, 16, 32


class StageVerifier:
    def __init__(self, param_sizes: Sequence[int], device, *, history: int = 1000, warmup: int = 20,
                 z_decision: float = 2.5, exclude_current: bool = True, max_quarantine: int = 2,
                 ema_beta: float = 0.8, symmetric_consistency: bool = True, quarantine: bool = True,
                 output_detection: bool = True, gradient_verification: bool = True,
                 consistency_tolerance: float = 2.0, deviation_deadzone: float = 0.25,
                 robust_baseline="detrend", baseline_window: int = 64, serialize_streams: bool = False,
                 features: str = "targeted", z_grad: float = 8.0, z_out: float = 8.0, sign_flip_cos: float = -0.7,
                 early_gate: bool = False):
        """``consistency_tolerance`` / ``deviation_deadzone`` make the trust metrics tolerate the
        legitimate drift of training (gradient norms routinely move 2x within a few steps early in
        training): a norm ratio r scores min(1, tol * min(r, 1/r)), an output deviation d scores
        max(0, d - dz) / (1 - dz).  tol=1, dz=0 gives the reference formulas exactly."""
        self.tol = float(consistency_tolerance)
        self.deadzone = float(deviation_deadzone)
        self.device = torch.device(device)
        self.output_detection = output_detection
        self.gradient_verification = gradient_verification
        self.quarantine = quarantine
        self.symmetric = symmetric_consistency
        self.beta = ema_beta
        self.warmup = warmup
        self.features = features
        if features == "reference":
            # the reference's decision rule: mean |z| over the 17 gradient / 12 output statistics
            kw = dict(history=history, warmup=warmup, z_decision=z_decision, exclude_current=exclude_current,
                      max_quarantine=max_quarantine, robust=robust_baseline, window=baseline_window)
            self.out_det = S.DeviceZScore(12, self.device, **kw)
            self.grad_det = S.DeviceZScore(17, self.device, **kw)
        else:
            # targeted: a few scale-free signals an attack must move — log gradient norm, log of
            # the largest per-parameter norm, log element std; output mean, log std, log |max| —
            # each against a detrended median / MAD baseline (the drift of learning), decision on
            # the largest |z|, scale floored at 5 % per step.  The cosine to the EMA reference
            # gradient is too autocorrelated for a z-score (it swings from -0.2 to 0.97 within a
            # few clean steps after a loss spike, MI355X trace r2): sign flips are caught by an
            # absolute rule instead (mean cosine < sign_flip_cos once the baseline is warm).  -0.7:
            # clean ResNet-50 gradients at micro-batch 8 dip below -0.4 against their EMA (the r2
            # attack-config trace: 13 false gradient flags at |z| < 3), a flipped gradient that
            # follows a real descent direction lands near -1
            # ``early_gate``: see ops.stats.DeviceZScore (set for verifiers built by a re-plan)
            kw = dict(history=history, warmup=warmup, exclude_current=exclude_current,
                      max_quarantine=max_quarantine, robust=robust_baseline, window=baseline_window,
                      agg="max", rel_floor=0.0, abs_floor=0.05, early_gate=early_gate)
            self.out_det = S.DeviceZScore(3, self.device, z_decision=z_out, **kw)
            self.grad_det = S.DeviceZScore(3, self.device, z_decision=z_grad, **kw)
        self.sign_flip_cos = float(sign_flip_cos)
        # the median / quartile histograms feed only the reference feature set (all 17 / 12
        # statistics); the targeted detectors never read them, so they are not computed
        self._quantiles = features == "reference"
        self.grad_stats = S.FlatGradStats(param_sizes, self.device) if len(param_sizes) else None
        self.sumsq = S.FlatSumSq(param_sizes, self.device)
        self.S = len(param_sizes)
        z = lambda *shape: torch.zeros(*shape, dtype=torch.float32, device=self.device)  # noqa: E731
        self.out_stats = z(13)
        self.out_mu, self.out_sd, self.out_n = z(1), z(1), z(1)
        self.norm_ema = z(max(self.S, 1))
        self.clip_w = torch.ones(max(self.S, 1), dtype=torch.float32, device=self.device)
        self.norm_n = z(1)
        self.ctrl = z(2)
        self.ctrl[0:1].fill_(1.0)
        self.digest = z(DIGEST)
        self._have_out = False
        self._skip_grad_once = False
        # ``serialize_streams`` (debug): run the statistics on the compute stream instead of the side
        # stream; with identical inputs the digests must match the overlapped run bit for bit (an
        # ordering bug between the two streams shows up as a difference; tests/test_kernels_gpu.py)
        self.side = (torch.cuda.Stream(self.device)
                     if self.device.type == "cuda" and not serialize_streams else None)

    # ---------------------------------------------------------------- output path
    def observe_output(self, y: torch.Tensor):
        """Queue statistics of a stage output (call once per step, e.g. for micro-batch 0)."""
        if not self.output_detection:
            return
        if self.side is not None:
            cur = torch.cuda.current_stream(self.device)
            self.side.wait_stream(cur)
            with torch.cuda.stream(self.side):
                S.tensor_stats(y.detach(), with_quantiles=self._quantiles, out=self.out_stats)
            y.record_stream(self.side)
        else:
            self.out_stats.copy_(S.tensor_stats(y.detach(), with_quantiles=self._quantiles))
        self._have_out = True

    # ---------------------------------------------------------------- gradient path + digest
    @property
    def verify_on(self) -> bool:
        return self.output_detection or self.gradient_verification

    @torch.no_grad()
    def grad_ready(self, flat_grad: torch.Tensor, seg_runs):
        """Segments (parameters) whose gradient is final for this step: run their K3 partial pass
        now, on the side stream after the compute stream's current point (overlaps the rest of
        the backward).  ``finish_step`` completes the pass."""
        if self.grad_stats is None or not self.verify_on or not flat_grad.is_cuda:
            return
        cur = torch.cuda.current_stream(self.device)
        stream = self.side if self.side is not None else cur
        if self.side is not None:
            self.side.wait_stream(cur)
        from ..ops.side_stream import wait_wgrad   # weight gradients may run on their own stream
        wait_wgrad(stream, self.device)
        for lo, hi in seg_runs:
            c0, c1 = self.grad_stats.chunk_range_of(lo, hi)
            self.grad_stats.partial(flat_grad, c0, c1, stream=stream)

    @torch.no_grad()
    def finish_step(self, flat_grad: Optional[torch.Tensor], loss: Optional[torch.Tensor],
                    host_metrics: Sequence[float], attack_truth: bool, stage_id: int) -> torch.Tensor:
        """Run detection on this step's signals and fill the digest row (device)."""
        if self.side is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.side)
        if VERIFY_FUSED and self.device.type == "cuda":
            return self._finish_fused(flat_grad, loss, host_metrics, attack_truth, stage_id)
        d = self.digest
        d.zero_()
        # scalar writes into device tensors go through fill_ (a kernel): `d[i] = 1.0` is a blocking
        # pageable host-to-device copy that drained the whole backward before the step tail
        # (HIP API trace: a 94 ms hipMemcpyWithStream per step, scripts/sync_probe.py)
        d[D_PRESENT:D_PRESENT + 1].fill_(1.0)
        d[D_STAGE:D_STAGE + 1].fill_(float(stage_id))
        if loss is not None:
            d[D_LOSS] = loss.detach().float().reshape(())
        # ---- output anomaly
        if self.output_detection and self._have_out:
            res = self.out_det.observe(self._out_features())
            d[D_OUT_FLAG] = res[0]
            d[D_OUT_Z] = res[1]
            d[D_OUT_CONF] = res[2]
            mu, sd = self.out_stats[0:1], self.out_stats[1:2]
            d[D_OUT_MEAN] = mu[0]
            d[D_OUT_STD] = sd[0]
            ready = (self.out_n >= self.warmup).float()
            dev = torch.clamp((torch.abs(mu - self.out_mu) + torch.abs(sd - self.out_sd)) /
                              (2.0 * torch.clamp(self.out_sd, min=1e-12)), max=1.0)
            dev = torch.clamp(dev - self.deadzone, min=0.0) / (1.0 - self.deadzone)
            d[D_METRICS + 0] = (dev * ready)[0]
            keep = 1.0 - res[0:1]  # do not fold flagged observations into the baseline
            first = (self.out_n == 0).float()
            b = self.beta * (1 - first) + 0.0 * first
            self.out_mu.copy_(keep * (b * self.out_mu + (1 - b) * mu) + (1 - keep) * self.out_mu)
            self.out_sd.copy_(keep * (b * self.out_sd + (1 - b) * sd) + (1 - keep) * self.out_sd)
            self.out_n.add_(keep)
            d[D_NONFINITE] += self.out_stats[12]
        # ---- gradient verification
        gflag = None
        bare = not self.verify_on
        if bare and self.grad_stats is not None and flat_grad is not None:
            # verification off: no statistics, quantiles or reference — only the clipping norm
            d[D_GRAD_SUMSQ] = self.sumsq.compute(flat_grad, self.clip_w)[0]
            d[D_METRICS + 1:D_METRICS + 2].fill_(1.0)
        elif self.grad_stats is not None and flat_grad is not None:
            g = self.grad_stats.compute(flat_grad, with_quantiles=self._quantiles)
            Sn = self.S
            norms = g[18:18 + Sn]
            sumsq = (norms * norms * self.clip_w[:Sn]).sum()
            d[D_GRAD_L2] = g[10]
            d[D_GRAD_COS] = g[16]
            d[D_NONFINITE] += g[17]
            if self.gradient_verification and self._skip_grad_once:
                self._skip_grad_once = False   # baselines restored without the EMA reference
            elif self.gradient_verification:
                res = self.grad_det.observe(self._grad_features(g))
                gflag = res[0:1]
                if self.features != "reference":
                    # sign flip: the gradient points against its own recent history
                    warm = (self.norm_n >= self.warmup).float()
                    gflag = torch.maximum(gflag, (g[16:17] < self.sign_flip_cos).float() * warm)
                d[D_GRAD_FLAG] = gflag[0]
                d[D_GRAD_Z] = res[1]
                d[D_GRAD_CONF] = res[2]
            ready = (self.norm_n >= self.warmup).float()
            r = norms / torch.clamp(self.norm_ema[:Sn], min=1e-30)
            if self.symmetric:
                sc = torch.minimum(r, 1.0 / torch.clamp(r, min=1e-30))
            else:
                sc = torch.clamp(r, max=1.0)
            sc = torch.clamp(sc * self.tol, max=1.0)
            valid = (self.norm_ema[:Sn] > 0).float()
            cons = (sc * valid).sum() / torch.clamp(valid.sum(), min=1.0)
            d[D_METRICS + 1] = ready[0] * cons + (1 - ready[0]) * 1.0
            keep = 1.0 - (gflag if gflag is not None else torch.zeros(1, device=self.device))
            first = (self.norm_n == 0).float()
            b = self.beta * (1 - first)
            self.norm_ema[:Sn].copy_(keep * (b * self.norm_ema[:Sn] + (1 - b) * norms) + (1 - keep) * self.norm_ema[:Sn])
            self.norm_n.add_(keep)
        else:
            d[D_METRICS + 1:D_METRICS + 2].fill_(1.0)
        # ---- host-side runtime metrics (latency, utilization, error, uptime), one step lagged
        hm = torch.tensor(list(host_metrics), dtype=torch.float32).pin_memory() \
            if self.device.type == "cuda" else torch.tensor(list(host_metrics), dtype=torch.float32)
        d[D_METRICS + 2:D_METRICS + 6].copy_(hm, non_blocking=True)
        # error rate metric: any non-finite value this step counts as an error
        d[D_METRICS + 4] = torch.clamp(d[D_METRICS + 4] + (d[D_NONFINITE] > 0).float(), max=1.0)
        d[D_ATTACK_TRUTH:D_ATTACK_TRUTH + 1].fill_(1.0 if attack_truth else 0.0)
        # ---- optimizer control block: quarantine flagged gradients on device
        if self.quarantine and gflag is not None:
            self.ctrl[1:2].copy_(torch.maximum(gflag, (d[D_NONFINITE:D_NONFINITE + 1] > 0).float()))
        else:
            self.ctrl[1:2].fill_(0.0)
        # clipping norm contribution: the gradient this stage will actually apply (a quarantined
        # update is skipped, so it must not shrink the honest stages' updates through the clip scale)
        if self.grad_stats is not None and flat_grad is not None and not bare:
            d[D_GRAD_SUMSQ] = sumsq * (1.0 - self.ctrl[1])
        self._have_out = False
        return d

    def _finish_fused(self, flat_grad, loss, host_metrics, attack_truth: bool, stage_id: int) -> torch.Tensor:
        """finish_step on the GPU in 2-5 launches: statistics final pass, detector features, the two
        detectors, and csrc/stats.hip verify_finish_kernel for everything else (same arithmetic as
        the torch form below; tests/test_kernels_gpu.py compares the two)."""
        from ..ops import _lib
        from ..ops._lib import ptr, stream_ptr
        if not getattr(StageVerifier, "_args_checked", False):
            n = int(_lib.lib().tdl_verify_args_bytes())
            if n != ctypes.sizeof(_FinishArgs):
                raise RuntimeError(f"VerifyFinishArgs layout mismatch: native {n} vs ctypes {ctypes.sizeof(_FinishArgs)}")
            StageVerifier._args_checked = True
        dev = self.device
        out_on = bool(self.output_detection and self._have_out)
        bare = not self.verify_on
        g = None
        grad_mode = 0
        sumsq_bare = None
        if bare and self.grad_stats is not None and flat_grad is not None:
            grad_mode = 1
            sumsq_bare = self.sumsq.compute(flat_grad, self.clip_w)
        elif self.grad_stats is not None and flat_grad is not None:
            grad_mode = 2
            g = self.grad_stats.compute(flat_grad, with_quantiles=self._quantiles)
        gdet = grad_mode == 2 and self.gradient_verification and not self._skip_grad_once
        if grad_mode == 2 and self.gradient_verification and self._skip_grad_once:
            self._skip_grad_once = False   # baselines restored without the EMA reference
        targeted = self.features != "reference"
        if out_on or gdet:
            if targeted:
                fb = getattr(self, "_feat_buf", None)
                if fb is None:
                    fb = self._feat_buf = torch.zeros(6, dtype=torch.float32, device=dev)
                _lib.call("tdl_verify_features", ptr(self.out_stats if out_on else None), ptr(g if gdet else None),
                          ptr(fb[0:3]), ptr(fb[3:6]), stream_ptr(dev))
                of, gf = fb[0:3], fb[3:6]
            else:
                of, gf = self.out_stats[:12], (g[:17] if g is not None else None)
        ores = self.out_det.observe(of) if out_on else None
        gres = self.grad_det.observe(gf) if gdet else None
        if loss is not None:
            lf = getattr(self, "_loss_buf", None)
            if lf is None:
                lf = self._loss_buf = torch.zeros(1, dtype=torch.float32, device=dev)
            lf.copy_(loss.detach().reshape(1))
        hm = [float(v) for v in host_metrics][:4] + [0.0] * max(0, 4 - len(host_metrics))
        a = _FinishArgs(
            d=self.digest.data_ptr(), loss=lf.data_ptr() if loss is not None else 0, stage_id=int(stage_id),
            out_on=int(out_on), out_res=ores.data_ptr() if ores is not None else 0,
            out_stats=self.out_stats.data_ptr(), out_mu=self.out_mu.data_ptr(), out_sd=self.out_sd.data_ptr(),
            out_n=self.out_n.data_ptr(), warmup=float(self.warmup), deadzone=float(self.deadzone),
            beta=float(self.beta), grad_mode=grad_mode,
            sumsq_bare=sumsq_bare.data_ptr() if sumsq_bare is not None else 0,
            g=g.data_ptr() if g is not None else 0, S=int(self.S), clip_w=self.clip_w.data_ptr(), gdet=int(gdet),
            grad_res=gres.data_ptr() if gres is not None else 0, targeted=int(targeted),
            sign_flip_cos=float(self.sign_flip_cos), norm_ema=self.norm_ema.data_ptr(),
            norm_n=self.norm_n.data_ptr(), tol=float(self.tol), symmetric=int(bool(self.symmetric)),
            hm0=hm[0], hm1=hm[1], hm2=hm[2], hm3=hm[3], truth=int(bool(attack_truth)),
            quarantine=int(bool(self.quarantine)), ctrl=self.ctrl.data_ptr())
        _lib.call("tdl_verify_finish", ctypes.byref(a), stream_ptr(dev))
        self._have_out = False
        return self.digest

    def _grad_features(self, g: torch.Tensor) -> torch.Tensor:
        if self.features == "reference":
            return g[:17]
        lg = lambda v: torch.log(torch.clamp(v, min=1e-30))  # noqa: E731
        return torch.stack([lg(g[10]), lg(g[15]), lg(g[1])])

    def _out_features(self) -> torch.Tensor:
        o = self.out_stats
        if self.features == "reference":
            return o[:12]
        return torch.stack([o[0], torch.log(torch.clamp(o[1], min=1e-30)), torch.log(torch.clamp(o[11], min=1e-30))])

    def set_clip_weights(self, weights: Sequence[float]):
        """Per-parameter weights (1 = counted, 0 = counted on another stage) for the digest's
        clipping sum of squares."""
        if len(weights):
            self.clip_w[:len(weights)].copy_(torch.tensor(list(weights), dtype=torch.float32))

    def set_clip_scale(self, total_sumsq: torch.Tensor, max_norm: float):
        """ctrl[0] = min(1, max_norm / ||g||_global) from the all-gathered per-stage sumsq (device)."""
        if max_norm and max_norm > 0:
            tot = torch.sqrt(torch.clamp(total_sumsq, min=0.0))
            self.ctrl[0:1].copy_(torch.clamp(max_norm / (tot + 1e-6), max=1.0).reshape(1))
        else:
            self.ctrl[0:1].fill_(1.0)

    def adopt(self, other: "StageVerifier"):
        """Take over another verifier's detector state for the same parameters (a stage rebuilt
        around unchanged layers): baselines, EMAs and the EMA reference gradient of the cosine
        feature (without it the first cosine after a rebuild reads 1.0 and looks like an attack)."""
        self.load_state_dict(other.state_dict())
        self._skip_grad_once = False
        if self.grad_stats is not None and other.grad_stats is not None and other.grad_stats.ref is not None \
                and self.grad_stats.ref is not None and other.grad_stats.ref.shape == self.grad_stats.ref.shape:
            self.grad_stats.ref = other.grad_stats.ref.to(self.device)
            self.grad_stats.ref_valid = other.grad_stats.ref_valid

    def rewarm(self):
        """After a re-plan: the detectors keep their most recent baseline entries but re-enter the
        early-gated warm-up (only gross outliers flag until the baseline has refilled)."""
        self.out_det.rewarm()
        self.grad_det.rewarm()

    def state_dict(self):
        return {k: v.detach().cpu() for k, v in {
            "out_ring": self.out_det.ring, "out_state": self.out_det.state,
            "grad_ring": self.grad_det.ring, "grad_state": self.grad_det.state,
            "out_mu": self.out_mu, "out_sd": self.out_sd, "out_n": self.out_n,
            "norm_ema": self.norm_ema, "norm_n": self.norm_n}.items()}

    def load_state_dict(self, sd):
        for k, t in (("out_ring", self.out_det.ring), ("out_state", self.out_det.state),
                     ("grad_ring", self.grad_det.ring), ("grad_state", self.grad_det.state),
                     ("out_mu", self.out_mu), ("out_sd", self.out_sd), ("out_n", self.out_n),
                     ("norm_ema", self.norm_ema), ("norm_n", self.norm_n)):
            if k in sd and sd[k].shape == t.shape:
                t.copy_(sd[k])
        # the EMA reference gradient is not checkpointed: its first cosine after a load reads 1.0,
        # so that one gradient observation is not scored against the restored baseline
        self._skip_grad_once = True
