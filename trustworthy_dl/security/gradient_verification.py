"""``GradientVerifier`` — per-stage gradient validity check.

The reference imports it (distributed_trainer.py:21, 81) and calls
``verify_gradients(grads, node_id, step) -> bool`` (distributed_trainer.py:199-205) but never
ships it.  Host API: a thin wrapper over ``AttackDetector.detect_gradient_poisoning`` (same
signature, attack_detector.py:109-141).  The training engine uses the device-resident
equivalent, ``StageVerifier`` (security/stage_verifier.py), which fuses the same statistics
into one segmented kernel and decides on device.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from .attack_detection import AttackDetector


class GradientVerifier:
    def __init__(self, detector: Optional[AttackDetector] = None, **detector_kwargs):
        self.detector = detector if detector is not None else AttackDetector(**detector_kwargs)
        self.verified = 0
        self.rejected = 0

    def verify_gradients(self, gradients: Sequence[torch.Tensor], node_id: int, step: int,
                         ground_truth: Optional[bool] = None) -> bool:
        """True if the gradients look benign, False if they are flagged as poisoned."""
        flagged = self.detector.detect_gradient_poisoning(list(gradients), node_id, step, ground_truth)
        if flagged:
            self.rejected += 1
        else:
            self.verified += 1
        return not flagged

    def statistics(self):
        return {"verified": self.verified, "rejected": self.rejected,
                **self.detector.get_detection_statistics()}
