"""Backward-pass audit primitives: gradient sketches and exact tensor hashes.

The reference's gradient check is a z-score over host statistics (attack_detector.py:109-141) that
cannot see a sign-flipped gradient (its F1 is 0.0) and its Byzantine check
compares outputs of DIFFERENT stages (attack_detector.py:143-162, 225-239).  Here the backward is
audited the way the forward is (parallel/pipeline.py ``_audit``): by recomputation.

* ``GradSketch`` — K random-sign projections of a sampled subset of a stage's flat fp32 gradient:
  from every block of ``block`` elements a window of ``win`` elements at a per-step offset (so each
  sketch reads ~1/16 of the buffer in whole cache lines), times a fixed +-1 pattern.  Linear, so
  the sketch of one micro-batch's weight-gradient contribution is the difference of two running
  sketches taken around its backward.  A stage COMMITS the running sketch after every
  micro-batch's backward and the sketch of the gradient it finally applies; its auditor recomputes
  one privately chosen micro-batch's backward and compares that contribution's sketch, and every
  rank checks that the applied gradient equals the sum of the committed contributions (a gradient
  rewritten between backward and optimizer — scaled, noised, zeroed or sign-flipped — fails this
  deterministically).  Blocks that hold a tied weight (whose gradient the tied all-reduce adds to)
  carry zero signs.
* ``hash2`` — an exact 32-bit fold of ``ops.stats.checksum`` (float64 sum / sum of squares /
  position-weighted sum), split into two 16-bit halves that an fp32 digest row carries exactly.

The sampling offset and the sign patterns are public (derived from the job seed, the step and the
stage's layer range); an adaptive adversary that knows them could hide a perturbation in the
unsampled coordinates — the simulated attacker (attacks/adversarial_attacks.py) does not.
"""
from __future__ import annotations

import hashlib
from typing import Iterable, Optional, Sequence, Tuple

import torch

from ..ops import stats as dstats

K_SKETCH = 2


def _block_for(n: int) -> int:
    b = 4096
    while b > 64 and n < 64 * b:
        b //= 2
    return b


class GradSketch:
    def __init__(self, numel: int, device, seed: int, masked: Iterable[Tuple[int, int]] = ()):
        self.numel = int(numel)
        self.block = _block_for(self.numel)
        self.win = self.block // 16
        self.nblk = self.numel // self.block
        g = torch.Generator().manual_seed(int(seed) & 0x7FFFFFFFFFFFFFFF)
        signs = torch.randint(0, 2, (K_SKETCH, max(self.nblk, 1), self.win), generator=g).float() * 2.0 - 1.0
        if self.nblk == 0:
            signs.zero_()
        # elements of a tied weight do not count: whole blocks get zero signs, a block that the
        # tied range only partly covers keeps its signs and an element mask (subtracted per call)
        part: dict = {}
        for lo, hi in masked:
            b0, b1 = lo // self.block, min(self.nblk, (hi + self.block - 1) // self.block)
            for bb in range(b0, b1):
                s0, s1 = bb * self.block, (bb + 1) * self.block
                if lo <= s0 and hi >= s1:
                    signs[:, bb, :] = 0.0
                    part.pop(bb, None)
                elif bb < self.nblk:
                    m = part.setdefault(bb, torch.zeros(self.block))
                    m[max(lo, s0) - s0:min(hi, s1) - s0] = 1.0
        self.signs = signs.to(device)
        self.partial = [(bb, m.to(device)) for bb, m in sorted(part.items()) if float(signs[:, bb].abs().sum()) > 0]

    def offset(self, seed: int, step: int) -> int:
        h = hashlib.blake2b(f"{seed}:gsk:{step}".encode(), digest_size=4).digest()
        return int.from_bytes(h, "little") % (self.block - self.win + 1)

    @torch.no_grad()
    def __call__(self, g: torch.Tensor, off: int) -> torch.Tensor:
        """[K] fp32 sketch of the flat gradient ``g`` (device, no host sync)."""
        if self.nblk == 0:
            return torch.zeros(K_SKETCH, dtype=torch.float32, device=g.device)
        v = g[: self.nblk * self.block].view(self.nblk, self.block)[:, off:off + self.win]
        out = (self.signs * v.unsqueeze(0)).sum(dim=(1, 2))
        for bb, m in self.partial:
            out = out - (self.signs[:, bb, :] * (v[bb] * m[off:off + self.win]).unsqueeze(0)).sum(-1)
        return out


def sketch_mismatch(seen: torch.Tensor, ref: torch.Tensor, tol: float, floor: Optional[torch.Tensor] = None):
    """(flag, relative error) of two [K] sketches, device tensors."""
    scale = ref.abs().amax()
    if floor is not None:
        scale = torch.maximum(scale, floor)
    err = (seen - ref).abs().amax() / scale.clamp_min(1e-20)
    err = torch.nan_to_num(err, nan=1e30, posinf=1e30)
    return (err > tol).float().reshape(1), err.reshape(1)


@torch.no_grad()
def hash2(x: torch.Tensor) -> torch.Tensor:
    """Exact 32-bit hash of a tensor's bytes as two fp32 values in [0, 65536) (device)."""
    return fold_hash(dstats.checksum(x.reshape(-1)))


def fold_hash(c: torch.Tensor) -> torch.Tensor:
    bits = c.double().contiguous().view(torch.int64)
    h = torch.zeros((), dtype=torch.int64, device=c.device)
    for i in range(bits.numel()):
        h = (h * 1000003) ^ bits[i]
    h = h ^ (h >> 32)
    h = h & 0xFFFFFFFF
    return torch.stack([(h & 0xFFFF).float(), ((h >> 16) & 0xFFFF).float()])


def tied_ranges(flat, tied_ids: Sequence[int]):
    """Flat-buffer ranges of the parameters in ``tied_ids``."""
    ids = set(tied_ids)
    return [(o, o + n) for q, o, n in zip(flat.params, flat.offsets, flat.sizes) if id(q) in ids]
