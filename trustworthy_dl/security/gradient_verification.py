"""``GradientVerifier`` — per-node gradient validity check.

The reference imports it (distributed_trainer.py:21, 81) and calls
``verify_gradients(grads, node_id, step) -> bool`` (distributed_trainer.py:199-205) but never
ships it (phantom).  SURVEY §2 names the intended behaviour — a per-tensor norm +
cosine-vs-reference + z-score check — which is what this class does, on two paths:

* device (GPU gradients): one ``StageVerifier`` per node in gradient-only mode.  The node's
  gradient list is packed into a persistent flat fp32 buffer (one fused copy), the segmented K3
  pass (csrc/stats.hip: per-parameter norms, moments, cosine against the node's EMA reference
  gradient, non-finite count) and the K4 z-score decision run on device, and only the 3-float
  verdict (flag, |z|, confidence) crosses to the host — the sync the bool-returning API implies.
* host (CPU gradients): ``AttackDetector.detect_gradient_poisoning`` (attack_detector.py:109-141),
  the reference's statistics with its z-score rule.

The training engine does not call this class per step: ``parallel/pipeline.py`` drives the same
``StageVerifier`` asynchronously from autograd hooks (no host sync in the step).  This is the
reference-shaped synchronous API for users who verify gradient lists themselves.
"""
from __future__ import annotations

import time
from collections import defaultdict, deque
from typing import Deque, Dict, List, Optional, Sequence

import torch

from .attack_detection import AttackDetectionResult, AttackDetector, AttackType
from .stage_verifier import D_GRAD_CONF, D_GRAD_FLAG, D_GRAD_L2, D_GRAD_COS, D_GRAD_Z, StageVerifier


class _NodeState:
    """Device verifier + flat gradient buffer of one node (rebuilt if its parameter shapes change)."""

    def __init__(self, sizes: List[int], device, **kw):
        self.sizes = sizes
        self.flat = torch.zeros(sum(sizes), dtype=torch.float32, device=device)
        self.verifier = StageVerifier(sizes, device, output_detection=False, gradient_verification=True,
                                      quarantine=False, **kw)


class GradientVerifier:
    def __init__(self, detector: Optional[AttackDetector] = None, *, warmup: int = 10, z_grad: float = 8.0,
                 sign_flip_cos: float = -0.7, history: int = 1000, **detector_kwargs):
        self.detector = detector if detector is not None else AttackDetector(**detector_kwargs)
        self.verified = 0
        self.rejected = 0
        self._dev_kw = dict(warmup=warmup, z_grad=z_grad, sign_flip_cos=sign_flip_cos, history=history)
        self._nodes: Dict[int, _NodeState] = {}
        self.history: Dict[int, Deque[dict]] = defaultdict(lambda: deque(maxlen=history))

    # ---------------------------------------------------------------- public API
    def verify_gradients(self, gradients: Sequence[torch.Tensor], node_id: int, step: int,
                         ground_truth: Optional[bool] = None) -> bool:
        """True if the gradients look benign, False if they are flagged as poisoned."""
        grads = [g for g in gradients if g is not None]
        if grads and grads[0].is_cuda:
            rec = self._verify_device(grads, node_id, step)
            flagged = rec["flagged"]
            # the detector's counters (detections, precision / recall ground truth) cover both paths
            res = AttackDetectionResult(flagged, AttackType.GRADIENT_POISONING if flagged else None,
                                        rec["confidence"], {"z": rec["z"], "path": "device"}, time.time(), node_id)
            self.detector._record(res, ground_truth, count_type=True)
        else:
            flagged = bool(self.detector.detect_gradient_poisoning(list(grads), node_id, step, ground_truth))
            rec = {"step": step, "flagged": flagged, "path": "host"}
        self.history[node_id].append(rec)
        if flagged:
            self.rejected += 1
        else:
            self.verified += 1
        return not flagged

    def statistics(self):
        return {"verified": self.verified, "rejected": self.rejected,
                "device_nodes": sorted(self._nodes),
                **self.detector.get_detection_statistics()}

    def node_history(self, node_id: int) -> List[dict]:
        return list(self.history.get(node_id, ()))

    def reset_node(self, node_id: int) -> None:
        """Forget a node's baselines (e.g. after its stage was rebuilt on another rank)."""
        self._nodes.pop(node_id, None)
        self.history.pop(node_id, None)

    # ---------------------------------------------------------------- device path
    @torch.no_grad()
    def _verify_device(self, grads: List[torch.Tensor], node_id: int, step: int) -> dict:
        sizes = [g.numel() for g in grads]
        st = self._nodes.get(node_id)
        if st is None or st.sizes != sizes or st.flat.device != grads[0].device:
            st = _NodeState(sizes, grads[0].device, **self._dev_kw)
            self._nodes[node_id] = st
        # one fused multi-tensor copy into the flat buffer (fp32: the statistics' input type)
        torch._foreach_copy_(list(torch.split(st.flat, sizes)), [g.detach().reshape(-1) for g in grads])
        v = st.verifier
        v.grad_ready(st.flat, [(0, len(sizes))])
        d = v.finish_step(st.flat, None, (0.0, 1.0, 0.0, 1.0), False, node_id)
        out = d[[D_GRAD_FLAG, D_GRAD_Z, D_GRAD_CONF, D_GRAD_L2, D_GRAD_COS]].cpu().tolist()
        return {"step": step, "flagged": out[0] > 0.5, "z": out[1], "confidence": out[2],
                "grad_norm": out[3], "cosine": out[4], "path": "device"}
