"""Backward-pass audit primitives: collision-resistant commitments, keyed sketches, contributions.

The reference's gradient check is a z-score over host statistics (attack_detector.py:109-141) that
cannot see a sign-flipped gradient (its F1 is 0.0), and its optimizer step
(distributed_trainer.py:197-205, :441-446) applies whatever gradient a node holds.  Here a stage's
gradient is bound by a commit / key / open protocol that its auditor verifies on data it hashes
itself (parallel/commitments.py, parallel/audit.py):

* ``merkle_roots`` — BLAKE2s Merkle root (256 bits) of a buffer's 32-bit words over a list of
  segments: leaves of 256 words (node_offset = leaf index, node_depth = 0), internal nodes over 32
  child digests (node_depth = level), one root per segment, then a combine node over the segment
  roots (node_depth = 255, last_node).  GPU: csrc/audit.hip, one thread per leaf / node, batched over
  the step's M contributions; CPU: ``hashlib.blake2s`` with the same node parameters, which is also
  the oracle of the GPU test.  Collision resistant, so an auditee cannot open a commitment to two
  different vectors (r5's additive mix32 hash had O(1) second preimages: scripts/lying_rank_before.py).
* ``keyed_sketch`` — K = 4 full-coverage random-sign projections whose signs come from a PRIVATE
  per-step key the auditor reveals only after it RECEIVED the commitments; linear, so the sketch of
  the applied gradient must equal the sum of the contributions' sketches.
* ``contrib_snap`` — after micro-batch i's weight gradients: c_i = g - prev, prev = g.
* ``GradSketch`` — K = 2 PUBLIC sketches of a 1/16 sample (job seed, step, layer range): only used
  to rank micro-batches for the targeted audit, never as a commitment (an adaptive adversary hides
  in its unsampled coordinates: tests/test_keyed_audit.py).
* ``hash_row`` — the first 128 bits of a root as eight exact fp32 16-bit halves for a digest row
  (cross-party comparisons: what one honest rank received vs what the auditee shipped).
"""
from __future__ import annotations

import hashlib
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch

K_SKETCH = 2
K_KEYED = 4
M32 = 0xFFFFFFFF
LEAF_WORDS = 256
FANOUT = 32
DIGEST_WORDS = 8
ROW_WORDS = 8          # digest-row floats per hash (128 bits as 16-bit halves)


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


# ====================================================================== BLAKE2s Merkle commitment
def _b2s(data, off: int, depth: int, last: bool = False) -> bytes:
    return hashlib.blake2s(data, digest_size=32, node_offset=off, node_depth=depth, last_node=last).digest()


def _tree_cpu(words: np.ndarray) -> bytes:
    """Root of one segment (uint32 words, >= 1): leaves, then >= 1 level of internal nodes."""
    buf = memoryview(np.ascontiguousarray(words, dtype="<u4").tobytes())
    lb = LEAF_WORDS * 4
    level = [_b2s(buf[j * lb:(j + 1) * lb], j, 0) for j in range((len(buf) + lb - 1) // lb)]
    depth = 1
    while True:
        level = [_b2s(b"".join(level[j * FANOUT:(j + 1) * FANOUT]), j, depth)
                 for j in range((len(level) + FANOUT - 1) // FANOUT)]
        depth += 1
        if len(level) == 1:
            return level[0]


def _combine_cpu(roots: Sequence[bytes]) -> bytes:
    return _b2s(b"".join(roots), 0, 255, last=True)


def _root_bytes_to_tensor(b: bytes) -> torch.Tensor:
    return torch.from_numpy(np.frombuffer(b, dtype="<u4").astype(np.int64)).to(torch.int32)


def merkle_roots_hashlib(x: torch.Tensor, segments: Sequence[Tuple[int, int]], batch: int = 1,
                         stride: int = 0) -> torch.Tensor:
    """The same roots with Python's hashlib.blake2s: the oracle of the native paths' tests."""
    w = x.reshape(-1).contiguous().view(torch.int32).numpy().view(np.uint32)
    segs = [(int(lo), int(hi)) for lo, hi in segments if hi > lo]
    out = [_root_bytes_to_tensor(_combine_cpu([_tree_cpu(w[y * stride + lo:y * stride + hi]) for lo, hi in segs]))
           for y in range(batch)]
    return torch.stack(out) if out else torch.zeros(0, DIGEST_WORDS, dtype=torch.int32)


def _merkle_host(flat: torch.Tensor, segs, batch: int, stride: int) -> torch.Tensor:
    """CPU tensors: the C++ host runtime (csrc/runtime/merkle.cpp, threads over leaves)."""
    import ctypes
    import os
    from ..runtime import native
    x = flat.contiguous()
    out = torch.empty(batch, DIGEST_WORDS, dtype=torch.int32)
    lo = (ctypes.c_longlong * max(1, len(segs)))(*[a for a, _ in segs])
    hi = (ctypes.c_longlong * max(1, len(segs)))(*[b for _, b in segs])
    threads = max(1, min(8, torch.get_num_threads(), os.cpu_count() or 1))
    rc = native.lib().tdl_host_merkle(ctypes.c_void_p(x.data_ptr()), stride, batch, lo, hi, len(segs), threads,
                                      ctypes.c_void_p(out.data_ptr()))
    if rc != 0:
        raise RuntimeError(f"tdl_host_merkle failed ({rc})")
    return out


@torch.no_grad()
def merkle_roots(x: torch.Tensor, segments: Sequence[Tuple[int, int]], batch: int = 1,
                 stride: Optional[int] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[batch, 8] int32 (raw uint32 bits) BLAKE2s Merkle roots of the 32-bit words of
    ``x.reshape(-1)[y * stride + lo : y * stride + hi]`` over ``segments``, y < batch (written into
    ``out`` when given: contiguous [batch, 8] int32).  Device tensors stay on the device (no host
    sync; runs on the current stream); identical bits on CPU and GPU."""
    flat = x.reshape(-1)
    if flat.element_size() != 4:
        raise ValueError("merkle_roots hashes 32-bit words")
    stride = int(stride if stride is not None else 0)
    segs = [(int(lo), int(hi)) for lo, hi in segments if hi > lo]
    if not flat.is_cuda:
        r = _merkle_host(flat, segs, batch, stride)
        if out is not None:
            out.copy_(r)
            return out
        return r
    from ..ops import _lib
    from ..ops._lib import ptr, stream_ptr
    dev = flat.device
    sp = stream_ptr(dev)
    if out is not None and (not out.is_contiguous() or tuple(out.shape) != (batch, DIGEST_WORDS)
                            or out.dtype != torch.int32 or out.device != dev):
        raise ValueError("out must be a contiguous [batch, 8] int32 tensor on the input's device")
    final = out if out is not None else torch.empty(batch, DIGEST_WORDS, dtype=torch.int32, device=dev)
    if not segs:
        final.copy_(_root_bytes_to_tensor(_combine_cpu([])).expand(batch, -1))
        return final
    nseg = len(segs)
    roots = final if nseg == 1 else torch.empty(batch, nseg, DIGEST_WORDS, dtype=torch.int32, device=dev)
    top_max = int(_lib.lib().tdl_b2s_top_max_in())
    for k, (lo, hi) in enumerate(segs):
        # leaves + level 1 in one launch, then (beyond ~8 M words) plain node levels, then the rest of
        # the tree in one workgroup per batch entry (with the final combine when there is one segment)
        nleaf = (hi - lo + LEAF_WORDS - 1) // LEAF_WORDS
        n = (nleaf + FANOUT - 1) // FANOUT
        cur = torch.empty(batch, n * DIGEST_WORDS, dtype=torch.int32, device=dev)
        _lib.call("tdl_b2s_leaves_l1", ptr(flat), stride, batch, lo, hi, ptr(cur), n * DIGEST_WORDS, sp)
        depth = 2
        while n > top_max:
            n_out = (n + FANOUT - 1) // FANOUT
            dst = torch.empty(batch, n_out * DIGEST_WORDS, dtype=torch.int32, device=dev)
            _lib.call("tdl_b2s_nodes", ptr(cur), n * DIGEST_WORDS, n, batch, FANOUT, depth, 0, ptr(dst),
                      n_out * DIGEST_WORDS, sp)
            cur, n, depth = dst, n_out, depth + 1
        if nseg == 1:
            _lib.call("tdl_b2s_top", ptr(cur), n * DIGEST_WORDS, n, batch, depth, 1, ptr(final), DIGEST_WORDS, sp)
        else:
            _lib.call("tdl_b2s_top", ptr(cur), n * DIGEST_WORDS, n, batch, depth, 0, ptr(roots[:, k]),
                      nseg * DIGEST_WORDS, sp)
    if nseg > 1:
        _lib.call("tdl_b2s_nodes", ptr(roots), nseg * DIGEST_WORDS, nseg, batch, nseg, 255, 1, ptr(final),
                  DIGEST_WORDS, sp)
    return final


def merkle_root(x: torch.Tensor, segments: Optional[Sequence[Tuple[int, int]]] = None) -> torch.Tensor:
    """[8] int32 Merkle root of one buffer (all of it when ``segments`` is None)."""
    if segments is None:
        segments = [(0, x.numel())]
    return merkle_roots(x, segments)[0]


def roots_differ(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """[1] float 1.0 where two roots (or [n, 8] root lists, compared row by row and OR-ed) differ."""
    return (a.to(b.device) != b).any().float().reshape(1)


def hash_row(root: torch.Tensor) -> torch.Tensor:
    """First 128 bits of a root as 8 fp32 values in [0, 65536) (exact) for a digest row."""
    h = root.reshape(-1)[:4].to(torch.int64) & M32
    return torch.stack([h & 0xFFFF, h >> 16], dim=1).reshape(-1).float()


def root_hex(root: torch.Tensor) -> str:
    return np.asarray(root.detach().cpu().to(torch.int64) & M32, dtype="<u4").tobytes().hex()


# ====================================================================== keyed sketch
def key_words(key: int) -> Tuple[int, int]:
    return int(key) & M32, (int(key) >> 32) & M32


@torch.no_grad()
def keyed_sketch(a: torch.Tensor, segments: Sequence[Tuple[int, int]], key: int,
                 b: Optional[torch.Tensor] = None, batch: Optional[int] = None,
                 stride: Optional[int] = None) -> torch.Tensor:
    """Keyed random-sign sketch of flat ``a`` (minus ``b``) over ``segments``: sign k of word j is
    bit 28 + k of mix(mix(j ^ k0) ^ k1), key = (k0, k1).  [K_KEYED] fp32, or [batch, K_KEYED] for
    ``a.reshape(-1)[y * stride + j]``.  Device, no host sync; fixed-order reductions, so the
    auditee's and the auditor's values of the same bits are identical."""
    single = batch is None
    batch = 1 if single else int(batch)
    stride = int(stride if stride is not None else 0)
    a = a.reshape(-1)
    k0, k1 = key_words(key)
    out = torch.zeros(batch, K_KEYED, dtype=torch.float32, device=a.device)
    if a.is_cuda:
        from ..ops import _lib
        from ..ops._lib import ptr, stream_ptr
        n = max((hi - lo for lo, hi in segments), default=0)
        per = int(_lib.lib().tdl_keyed_sketch_ws_floats(max(1, n)))
        ws = torch.empty(max(4, per * batch), dtype=torch.float32, device=a.device)
        for i, (lo, hi) in enumerate(segments):
            _lib.call("tdl_keyed_sketch", ptr(a), stride, batch, ptr(None if b is None else b.reshape(-1)), int(lo),
                      int(hi), k0, k1, ptr(ws), ptr(out), 1 if i else 0, stream_ptr(a.device))
        return out[0] if single else out
    bf = None if b is None else b.reshape(-1)
    for lo, hi in segments:
        j = torch.arange(lo, hi, dtype=torch.int64) & M32
        h = _mix32(_mix32(j ^ k0) ^ k1)
        signs = torch.stack([1.0 - 2.0 * ((h >> (28 + k)) & 1).float() for k in range(K_KEYED)])
        for y in range(batch):
            v = a[y * stride + lo:y * stride + hi].float()
            if bf is not None:
                v = v - bf[lo:hi].float()
            out[y] += (signs * v).sum(1)
    return out[0] if single else out


@torch.no_grad()
def seg_rel_err(a: torch.Tensor, ref: torch.Tensor, segments) -> torch.Tensor:
    """max |a - ref| / max |ref| over the segments (device scalar, no host sync, no n-sized
    temporaries on the GPU; NaN / inf -> 1e30)."""
    a, ref = a.reshape(-1), ref.reshape(-1)
    if not segments:
        return torch.zeros((), device=ref.device)
    if a.is_cuda:
        from ..ops import _lib
        from ..ops._lib import ptr, stream_ptr
        bits = torch.zeros(2, dtype=torch.int32, device=a.device)
        for lo, hi in segments:
            _lib.call("tdl_absdiff_max", ptr(a), ptr(ref), int(lo), int(hi), ptr(bits), stream_ptr(a.device))
        v = bits.view(torch.float32)
        num, den = v[0], v[1].clamp_min(1e-30)
    else:
        num = torch.stack([(a[lo:hi] - ref[lo:hi]).abs().amax() for lo, hi in segments]).amax()
        den = torch.stack([ref[lo:hi].abs().amax() for lo, hi in segments]).amax().clamp_min(1e-30)
    return torch.nan_to_num(num / den, nan=1e30, posinf=1e30)


@torch.no_grad()
def seg_sumsq(x: torch.Tensor, segments) -> torch.Tensor:
    """sum of squares over the segments (device scalar, no n-sized temporary)."""
    x = x.reshape(-1)
    if not segments:
        return torch.zeros((), device=x.device)
    return torch.stack([torch.linalg.vector_norm(x[lo:hi], 2).square() for lo, hi in segments]).sum()


@torch.no_grad()
def contrib_snap(g: torch.Tensor, prev: torch.Tensor, c: torch.Tensor) -> None:
    """c = g - prev; prev = g (one micro-batch's weight-gradient contribution, fp32)."""
    if g.is_cuda:
        from ..ops import _lib
        from ..ops._lib import ptr, stream_ptr
        _lib.call("tdl_contrib_snap", ptr(g), ptr(prev), ptr(c), g.numel(), stream_ptr(g.device))
        return
    torch.sub(g, prev, out=c)
    prev.copy_(g)


# ====================================================================== public sketch (targeting only)
def _block_for(n: int) -> int:
    b = 4096
    while b > 64 and n < 64 * b:
        b //= 2
    return b


class GradSketch:
    """K_SKETCH random-sign projections of a public 1/16 sample of a flat gradient (targeting)."""

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


def tied_ranges(flat, tied_ids: Sequence[int]):
    """Flat-buffer ranges of the parameters in ``tied_ids``."""
    ids = set(tied_ids)
    return [(o, o + n) for q, o, n in zip(flat.params, flat.offsets, flat.sizes) if id(q) in ids]

