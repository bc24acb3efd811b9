"""Adversary / fault injection: ``AttackConfig`` and ``AdversarialAttacker``.

The reference imports these (experiment_runner.py:23, 91-97, 157-160, 187-188, 231, 285, 598;
README.md:61) but never ships them.  Inferred API kept:
``AttackConfig(attack_types, target_nodes, intensity, start_step)``; ``activate_attacks()``,
``is_active()``, ``apply_attacks(batch, batch_idx)``, ``get_attack_statistics()``,
``get_final_statistics()``, ``cleanup()``.

Attacks act on *stages* through engine hooks, in place on device tensors via the Philox-seeded
injection kernel (csrc/attack.hip), and every injection is logged as ground truth so detection
precision / recall / F1 and time-to-detect are measured, not simulated (cf. the simulated curves
of experiment_runner.py:439-451):

* ``gradient_poisoning`` — the stage's accumulated gradient is scaled / noised / sign-flipped /
  zeroed before verification (``gradient_mode``);
* ``model_poisoning`` (param perturbation) — the stage's weights are multiplicatively perturbed;
* ``byzantine`` — the stage's output activations are tampered before they are sent downstream;
* ``byzantine_backward`` — the activation gradient the stage sends UPSTREAM (its input gradient)
  is tampered (sign flip + relative noise), the backward-pass counterpart of ``byzantine``;
* ``data_poisoning`` — labels are flipped and inputs perturbed in the batch (consumed by stage 0).

``micro_batches`` (k) restricts the per-micro-batch attacks to k of the step's M micro-batches
(chosen by the attacker's own per-step hash): ``byzantine`` / ``byzantine_backward`` tamper only
those, and ``gradient_poisoning`` then acts INSIDE the backward, on those micro-batches'
weight-gradient contributions (sign-flipped / scaled / zeroed / noised as ``gradient_mode`` says)
instead of on the step's accumulated gradient — the one-of-M adversary that a one-micro-batch
audit catches with probability k / M per step.  ``lie_integrity``: the target's engine reports a
passing weight-integrity check whatever it measured (a rank that lies about its own checksum).

``adaptive`` (gradient poisoning): the attacker knows everything public about the audit — the job
seed, the step, the stage's layer range, hence r4's public gradient sketch (its sampled window
offset and sign vectors; the engine hands it over as ``public_sketch_fn``) — and confines its
tamper to the coordinates that sketch does not sample, so the sketch of the tampered gradient
equals the clean one bit for bit.  r4's commitments passed it; the commit-then-reveal check
(exact hashes + keyed sketches under a key revealed after the commitment) catches it.
"""
from __future__ import annotations

import hashlib
import logging
import time
from collections import defaultdict
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np
import torch

from ..ops.attack import AttackMode, inject_

logger = logging.getLogger(__name__)

ATTACK_TYPES = ("gradient_poisoning", "model_poisoning", "byzantine", "byzantine_backward", "data_poisoning",
                "backdoor", "adversarial_input")
_GRAD_MODES = {"scale": AttackMode.SCALE, "noise": AttackMode.REL_NOISE, "sign_flip": AttackMode.SIGN_FLIP,
               "zero": AttackMode.ZERO, "additive_noise": AttackMode.NOISE}


@dataclass
class AttackConfig:
    attack_types: List[str] = field(default_factory=lambda: ["gradient_poisoning"])
    target_nodes: List[int] = field(default_factory=lambda: [1])
    intensity: float = 0.5
    start_step: int = 0
    end_step: Optional[int] = None
    probability: float = 1.0            # per-step, per-target attack probability
    gradient_mode: str = "scale"        # scale | noise | sign_flip | zero | additive_noise
    gradient_scale: Optional[float] = None   # default 1 + 18 * intensity (0.5 -> x10)
    param_noise: Optional[float] = None      # relative weight noise, default intensity
    activation_noise: Optional[float] = None  # relative activation noise, default 4 * intensity
    label_flip_fraction: Optional[float] = None  # default intensity
    micro_batches: Optional[int] = None  # tamper only this many of the step's micro-batches (None: all)
    lie_integrity: bool = False          # the target reports its weight-integrity check as passing
    adaptive: bool = False               # gradient tampers avoid everything the public sketch samples
    seed: int = 1234

    def grad_factor(self) -> float:
        return self.gradient_scale if self.gradient_scale is not None else 1.0 + 18.0 * self.intensity


class AdversarialAttacker:
    def __init__(self, config: AttackConfig):
        for t in config.attack_types:
            if t not in ATTACK_TYPES:
                raise ValueError(f"unknown attack type {t!r}; choose from {ATTACK_TYPES}")
        self.config = config
        self.active = False
        self.injections: List[Dict] = []          # ground-truth log
        self.detections: Dict[int, List[int]] = defaultdict(list)
        self.counts = defaultdict(int)
        self.outcomes = defaultdict(int)          # tp/fp/fn/tn from the engine's detector
        self.first_attack_step: Dict[int, int] = {}
        self.first_detect_step: Dict[int, int] = {}
        self.last_batch_truth: Dict[int, bool] = {}
        # set by the engine: node -> (public GradSketch, its per-step window offset) — public data
        self.public_sketch_fn = None
        self._gsnap = None

    # ---------------------------------------------------------------- activation
    def activate_attacks(self):
        self.active = True
        logger.warning("Attacks activated: %s on nodes %s", self.config.attack_types, self.config.target_nodes)

    def deactivate_attacks(self):
        self.active = False

    def is_active(self) -> bool:
        return self.active

    def _fires(self, kind: str, node: int, step: int) -> bool:
        c = self.config
        if not self.active or kind not in c.attack_types or node not in c.target_nodes:
            return False
        if step < c.start_step or (c.end_step is not None and step > c.end_step):
            return False
        if c.probability >= 1.0:
            return True
        h = hashlib.blake2b(f"{c.seed}:{kind}:{node}:{step}".encode(), digest_size=8).digest()
        return int.from_bytes(h, "little") / 2.0 ** 64 < c.probability

    def micro_fires(self, kind: str, node: int, step: int, micro: Optional[int], num_micro: Optional[int]) -> bool:
        """Does ``kind`` hit micro-batch ``micro`` of ``num_micro`` at this step?  With
        ``micro_batches = k`` the attacker tampers k micro-batches per step, picked by its own hash
        of (seed, node, step) — independent of the auditor's private choice."""
        if not self._fires(kind, node, step):
            return False
        k = self.config.micro_batches
        if k is None or micro is None or not num_micro or k >= num_micro:
            return True
        h = hashlib.blake2b(f"{self.config.seed}:micro:{kind}:{node}:{step}".encode(), digest_size=8).digest()
        rng = np.random.default_rng(int.from_bytes(h, "little"))
        return int(micro) in set(rng.choice(int(num_micro), size=int(k), replace=False).tolist())

    def per_micro_gradients(self) -> bool:
        """Gradient poisoning acts inside the backward (on k micro-batches' contributions)."""
        return self.config.micro_batches is not None and "gradient_poisoning" in self.config.attack_types

    def lies_about_integrity(self, node: int, step: int) -> bool:
        return self.config.lie_integrity and self.active and node in self.config.target_nodes

    def _log(self, kind: str, node: int, step: int, **info):
        self.injections.append({"type": kind, "node": node, "step": step, "timestamp": time.time(), **info})
        self.counts[kind] += 1
        self.first_attack_step.setdefault(node, step)

    def _seed(self, node: int, step: int) -> int:
        return (self.config.seed * 1_000_003 + node * 7919 + step) & 0xFFFFFFFFFFFF

    # ---------------------------------------------------------------- engine hooks
    def _grad_magnitude(self, g: torch.Tensor):
        c = self.config
        mode = _GRAD_MODES[c.gradient_mode]
        a = {AttackMode.SCALE: c.grad_factor(), AttackMode.REL_NOISE: 10.0 * c.intensity,
             AttackMode.SIGN_FLIP: 1.0, AttackMode.ZERO: 0.0, AttackMode.NOISE: c.intensity}[mode]
        if mode == AttackMode.NOISE:  # absolute noise scaled to the gradient's RMS
            a = float(c.intensity * 10.0 * g.float().pow(2).mean().sqrt().item() + 1e-12)
        return mode, a

    def _hide(self, node: int, delta: torch.Tensor) -> torch.Tensor:
        """``adaptive``: zero the tamper on every coordinate the public sketch reads (its sampled
        window in each block), so that sketch cannot see it at all."""
        if not self.config.adaptive or self.public_sketch_fn is None:
            return delta
        sk, off = self.public_sketch_fn(node)
        if sk is not None and sk.nblk > 0:
            delta[: sk.nblk * sk.block].view(sk.nblk, sk.block)[:, off:off + sk.win] = 0.0
        return delta

    def on_gradients(self, node: int, flat_grad: torch.Tensor, step: int) -> bool:
        if self.per_micro_gradients() or not self._fires("gradient_poisoning", node, step):
            return False
        mode, a = self._grad_magnitude(flat_grad)
        if self.config.adaptive:
            t = flat_grad.detach().clone()
            inject_(t, mode, a, self._seed(node, step), 0)
            flat_grad.add_(self._hide(node, t - flat_grad))
        else:
            inject_(flat_grad, mode, a, self._seed(node, step), 0)
        self._log("gradient_poisoning", node, step, mode=self.config.gradient_mode, magnitude=a,
                  adaptive=self.config.adaptive)
        return True

    # gradient poisoning inside the backward (``micro_batches`` set): the engine calls
    # before_micro_backward / after_micro_backward around each micro-batch's backward of the stage
    # (its weight-gradient contribution d = G_after - G_before), and the attack rewrites d in place
    def before_micro_backward(self, node: int, flat_grad: torch.Tensor, step: int, micro: int, num_micro: int):
        if self.per_micro_gradients() and self.micro_fires("gradient_poisoning", node, step, micro, num_micro):
            self._gsnap = (node, step, micro, flat_grad.detach().clone())

    def after_micro_backward(self, node: int, flat_grad: torch.Tensor, step: int, micro: int, num_micro: int) -> bool:
        snap = self._gsnap
        if snap is None or snap[:3] != (node, step, micro):
            return False
        self._gsnap = None
        before = snap[3]
        d = flat_grad - before
        mode, a = self._grad_magnitude(d)
        t = d.clone()
        inject_(t, mode, a, self._seed(node, step) + micro, 0)
        flat_grad.copy_(before + d + self._hide(node, t - d) if self.config.adaptive else before + t)
        self._log("gradient_poisoning", node, step, mode=self.config.gradient_mode, magnitude=a, micro=micro,
                  adaptive=self.config.adaptive)
        return True

    def on_input_grad(self, node: int, dx: torch.Tensor, step: int, micro: Optional[int] = None,
                      num_micro: Optional[int] = None) -> Optional[torch.Tensor]:
        """Byzantine backward: tamper the activation gradient the stage sends upstream."""
        if not self.micro_fires("byzantine_backward", node, step, micro, num_micro):
            return None
        a = self.config.activation_noise if self.config.activation_noise is not None else 4.0 * self.config.intensity
        out = dx.detach().clone().contiguous()
        inject_(out, AttackMode.REL_NOISE, a, self._seed(node, step) + (micro or 0), 0)
        inject_(out, AttackMode.SIGN_FLIP, 1.0)
        self._log("byzantine_backward", node, step, magnitude=a, micro=micro)
        return out

    def on_parameters(self, node: int, flat, step: int) -> bool:
        if not self._fires("model_poisoning", node, step):
            return False
        a = self.config.param_noise if self.config.param_noise is not None else self.config.intensity
        inject_(flat.master, AttackMode.REL_NOISE, a, self._seed(node, step), 0)
        if flat.data is not flat.master:
            flat.data.copy_(flat.master)
        self._log("model_poisoning", node, step, magnitude=a)
        return True

    def on_output(self, node: int, y: torch.Tensor, step: int, micro: Optional[int] = None,
                  num_micro: Optional[int] = None) -> Optional[torch.Tensor]:
        if not self.micro_fires("byzantine", node, step, micro, num_micro):
            return None
        a = self.config.activation_noise if self.config.activation_noise is not None else 4.0 * self.config.intensity
        yt = y.detach()
        if not yt.is_contiguous():
            return None
        # in place, before any consumer has read the activation (the producer saved none of it)
        inject_(yt, AttackMode.REL_NOISE, a, self._seed(node, step) + (micro or 0), 0)
        inject_(yt, AttackMode.SIGN_FLIP, 1.0)
        self._log("byzantine", node, step, magnitude=a, micro=micro)
        return y

    def apply_attacks(self, batch: Dict[str, torch.Tensor], batch_idx: int) -> Dict[str, torch.Tensor]:
        """Data poisoning on the batch (experiment_runner.py:187-188): label flipping + input noise.
        The poisoned data is consumed by stage 0, which is the ground-truth target."""
        self.last_batch_truth = {}
        c = self.config
        if not (self.active and "data_poisoning" in c.attack_types and batch_idx >= c.start_step
                and (c.end_step is None or batch_idx <= c.end_step)):
            return batch
        if c.probability < 1.0:
            h = hashlib.blake2b(f"{c.seed}:data:{batch_idx}".encode(), digest_size=8).digest()
            if int.from_bytes(h, "little") / 2.0 ** 64 >= c.probability:
                return batch
        frac = self.config.label_flip_fraction if self.config.label_flip_fraction is not None else self.config.intensity
        g = torch.Generator().manual_seed(self._seed(0, batch_idx))
        out = dict(batch)
        tgt = batch["target"].clone()
        mask = torch.rand(tgt.shape, generator=g) < frac
        hi = int(tgt.max()) + 1 if tgt.numel() else 1
        tgt[mask] = torch.randint(0, max(hi, 2), (int(mask.sum()),), generator=g)
        out["target"] = tgt
        x = batch["input"]
        if x.is_floating_point():
            out["input"] = x + torch.randn(x.shape, generator=g) * (4.0 * frac) * x.std()
        self._log("data_poisoning", 0, batch_idx, fraction=frac)
        self.last_batch_truth[0] = True
        return out

    # ---------------------------------------------------------------- detection bookkeeping
    def record_detection(self, node: int, step: int, detected: bool, truth: bool):
        key = ("tp" if truth else "fp") if detected else ("fn" if truth else "tn")
        self.outcomes[key] += 1
        if detected:
            self.detections[node].append(step)
            if truth:
                self.first_detect_step.setdefault(node, step)

    def detection_metrics(self) -> Dict[str, float]:
        tp, fp, fn, tn = (self.outcomes[k] for k in ("tp", "fp", "fn", "tn"))
        p = tp / (tp + fp) if tp + fp else 0.0
        r = tp / (tp + fn) if tp + fn else 0.0
        ttd = {n: self.first_detect_step[n] - self.first_attack_step[n]
               for n in self.first_detect_step if n in self.first_attack_step}
        return {"tp": tp, "fp": fp, "fn": fn, "tn": tn, "precision": p, "recall": r,
                "f1": 2 * p * r / (p + r) if p + r else 0.0,
                "time_to_detect_steps": ttd,
                "mean_time_to_detect_steps": float(np.mean(list(ttd.values()))) if ttd else None}

    def get_attack_statistics(self) -> Dict:
        return {"active": self.active, "total_injections": len(self.injections),
                "by_type": dict(self.counts), "target_nodes": list(self.config.target_nodes),
                **self.detection_metrics()}

    def get_final_statistics(self) -> Dict:
        s = self.get_attack_statistics()
        s["config"] = {k: (list(v) if isinstance(v, list) else v) for k, v in self.config.__dict__.items()}
        s["injections"] = self.injections[-1000:]
        return s

    def cleanup(self):
        self.active = False
        logger.info("AdversarialAttacker cleanup completed")
