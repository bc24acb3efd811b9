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

``GradSketch``'s sampling offset and sign patterns are public (derived from the job seed, the step
and the stage's layer range): an adaptive adversary that knows them hides a perturbation in the
unsampled coordinates or in the null space of the public signs (attacks/adversarial_attacks.py
``adaptive``; tests/test_keyed_audit.py shows it passes that sketch).  It now only ranks micro-batches
for the targeted audit.  The binding checks use

* ``word_hash`` — an EXACT, order-independent 64-bit hash of a buffer's 32-bit words
  (csrc/audit.hip): the running gradient after every micro-batch and the applied gradient are
  committed by hash, so a gradient rewritten between backward and optimizer fails bit-exactly, on
  every coordinate;
* ``keyed_sketch`` — K = 4 full-coverage random-sign projections whose signs come from a PRIVATE
  per-step key the auditor reveals only after the auditee's commitments were sent: the auditee
  answers with the keyed sketch of the audited micro-batch's committed contribution (the difference
  of two snapshots whose hashes it committed), the auditor compares it with the sketch of its
  recomputation.  A perturbation chosen before the key is known cannot avoid the signs.
"""
from __future__ import annotations

import hashlib
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import torch

from ..ops import stats as dstats

K_SKETCH = 2
K_KEYED = 4
M32 = 0xFFFFFFFF


def _mix32(x: torch.Tensor) -> torch.Tensor:
    """csrc/audit.hip mix32 on int64 tensors holding uint32 values (constants < 2^31: no overflow)."""
    x = x ^ (x >> 16)
    x = (x * 0x7feb352d) & M32
    x = x ^ (x >> 15)
    x = (x * 0x6c8e9cf5) & M32
    return x ^ (x >> 16)


def _segments(n: int, masked: Sequence[Tuple[int, int]] = ()) -> List[Tuple[int, int]]:
    """[0, n) minus the masked ranges, as sorted disjoint (lo, hi) segments."""
    segs, pos = [], 0
    for lo, hi in sorted((max(0, a), min(n, b)) for a, b in masked):
        if lo > pos:
            segs.append((pos, lo))
        pos = max(pos, hi)
    if pos < n:
        segs.append((pos, n))
    return segs


_pmix: Dict[Tuple[int, int, int], torch.Tensor] = {}


def _position_mix(lo: int, hi: int, seed: int) -> torch.Tensor:
    """CPU path: mix(j ^ seed) over [lo, hi) (one seed serves every commitment of a step)."""
    key = (lo, hi, seed)
    t = _pmix.get(key)
    if t is None:
        if len(_pmix) > 16:
            _pmix.clear()
        t = _pmix[key] = _mix32((torch.arange(lo, hi, dtype=torch.int64) & M32) ^ seed)
    return t


@torch.no_grad()
def word_hash(x: torch.Tensor, segments: Sequence[Tuple[int, int]], seed: int = 0,
              snapshot: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Exact 64-bit hash (int64 device tensor [1]) of the 32-bit words of flat ``x`` over
    ``segments`` (global word indices); with ``snapshot`` the same pass copies those words into it.
    No host sync.  Identical bits give identical hashes on CPU and GPU."""
    x = x.reshape(-1)
    if x.element_size() != 4:
        raise ValueError("word_hash works on 32-bit words")
    if out is None:
        out = torch.zeros(1, dtype=torch.int64, device=x.device)
    else:
        out.zero_()
    if x.is_cuda:
        from ..ops import _lib
        from ..ops._lib import ptr, stream_ptr
        for lo, hi in segments:
            _lib.call("tdl_word_hash", ptr(x), ptr(snapshot), int(lo), int(hi), int(seed) & M32, ptr(out),
                      stream_ptr(x.device))
        return out
    w = x.view(torch.int32).to(torch.int64) & M32
    tot = torch.zeros((), dtype=torch.int64)
    for lo, hi in segments:
        tot = tot + _mix32(w[lo:hi] ^ _position_mix(lo, hi, int(seed) & M32)).sum()
        if snapshot is not None:
            snapshot.reshape(-1)[lo:hi].copy_(x[lo:hi])
    out.copy_(tot.reshape(1))
    return out


def fold_hash64(h: torch.Tensor) -> torch.Tensor:
    """A ``word_hash`` as two fp32 values in [0, 65536) (its 32-bit fold) for a digest row."""
    h = h.reshape(())
    f = (h ^ (h >> 32)) & M32
    return torch.stack([(f & 0xFFFF).float(), ((f >> 16) & 0xFFFF).float()])


def key_words(key: int) -> Tuple[int, int]:
    return int(key) & M32, (int(key) >> 32) & M32


@torch.no_grad()
def keyed_sketch(a: torch.Tensor, segments: Sequence[Tuple[int, int]], key: int,
                 b: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[K_KEYED] fp32 keyed random-sign sketch of flat ``a`` (minus ``b``) over ``segments``: sign
    k of word j is bit 28 + k of mix(mix(j ^ k0) ^ k1), key = (k0, k1).  Device, no host sync."""
    a = a.reshape(-1)
    k0, k1 = key_words(key)
    out = torch.zeros(K_KEYED, dtype=torch.float32, device=a.device)
    if a.is_cuda:
        from ..ops import _lib
        from ..ops._lib import ptr, stream_ptr
        n = max((hi - lo for lo, hi in segments), default=0)
        ws = torch.empty(max(4, int(_lib.lib().tdl_keyed_sketch_ws_floats(max(1, n)))), dtype=torch.float32,
                         device=a.device)
        for i, (lo, hi) in enumerate(segments):
            _lib.call("tdl_keyed_sketch", ptr(a), ptr(None if b is None else b.reshape(-1)), int(lo), int(hi),
                      k0, k1, ptr(ws), ptr(out), 1 if i else 0, stream_ptr(a.device))
        return out
    bf = None if b is None else b.reshape(-1)
    for lo, hi in segments:
        j = torch.arange(lo, hi, dtype=torch.int64) & M32
        h = _mix32(_mix32(j ^ k0) ^ k1)
        v = a[lo:hi].float() if bf is None else a[lo:hi].float() - bf[lo:hi].float()
        for k in range(K_KEYED):
            s = 1.0 - 2.0 * ((h >> (28 + k)) & 1).float()
            out[k] += (s * v).sum()
    return out


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
        # elements of a tied weight do not count: every block a tied range touches gets zero signs
        # (a block only partly covered used to add the tied elements in one kernel and
        # subtract them in a second, so a tied all-reduce writing in between skewed the sketch)
        for lo, hi in masked:
            b0, b1 = lo // self.block, min(self.nblk, (hi + self.block - 1) // self.block)
            if b1 > b0:
                signs[:, b0:b1, :] = 0.0
        self.signs = signs.to(device)

    def offset(self, seed: int, step: int) -> int:
        h = hashlib.blake2b(f"{seed}:gsk:{step}".encode(), digest_size=4).digest()
        return int.from_bytes(h, "little") % (self.block - self.win + 1)

    @torch.no_grad()
    def __call__(self, g: torch.Tensor, off: int) -> torch.Tensor:
        """[K] fp32 sketch of the flat gradient ``g`` (device, no host sync)."""
        if self.nblk == 0:
            return torch.zeros(K_SKETCH, dtype=torch.float32, device=g.device)
        v = g[: self.nblk * self.block].view(self.nblk, self.block)[:, off:off + self.win]
        return (self.signs * v.unsqueeze(0)).sum(dim=(1, 2))


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
