"""Device statistics, detection and trust kernels (csrc/stats.hip) with CPU references.

Statistic vector layouts match ``security.attack_detection.TENSOR_STATS`` / ``GRAD_STATS``.
Quantiles on the GPU come from a 2048-bin histogram over [min, max] (error <= one bin width,
i.e. (max - min) / 2048); the CPU path is exact (numpy definitions).
"""
from __future__ import annotations

import ctypes
import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import ptr, stream_ptr

N_TENSOR_STATS = 12
N_GRAD_STATS = 17
NHIST = 2048
CHUNK = 1 << 13    # elements per partial-statistics block: >= 4 blocks per CU for a GPT-2-medium weight
REF_STRIDE = 8       # the EMA reference gradient is kept on one chunk in REF_STRIDE (csrc/stats.hip)

_ws_cache = {}


def _workspace(dev: torch.device, nbytes: int) -> torch.Tensor:
    """Persistent scratch of the statistics kernels, one per (device, current stream): two stages
    sharing a GPU (local mode) run their output statistics on their own side streams concurrently,
    and a per-device buffer let them overwrite each other's partials (flaky output mean / std in the
    digests: tests/test_engine_gpu.py serialized-vs-overlapped, 2 of 6 suite runs)."""
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    key = (idx, torch.cuda.current_stream(torch.device("cuda", idx)).cuda_stream)
    w = _ws_cache.get(key)
    if w is None or w.numel() < nbytes:
        w = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=dev)
        _ws_cache[key] = w
    return w


# ------------------------------------------------------------------ CPU reference
def _cpu_stats(x: torch.Tensor) -> torch.Tensor:
    from ..security.attack_detection import numpy_tensor_statistics, TENSOR_STATS
    arr = x.detach().float().reshape(-1).numpy()
    fin = np.isfinite(arr)
    st = numpy_tensor_statistics(arr[fin]) if fin.any() else {k: 0.0 for k in TENSOR_STATS}
    return torch.tensor([st[k] for k in TENSOR_STATS] + [float((~fin).sum())], dtype=torch.float32)


def tensor_stats(x: torch.Tensor, with_quantiles: bool = True, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """[13] float32: TENSOR_STATS + non-finite count.  Device-resident for GPU input."""
    if not x.is_cuda:
        return _cpu_stats(x)
    x = x.detach()
    if not x.is_contiguous():
        x = x.contiguous()
    code = _lib.DTYPE_CODE[x.dtype] if x.dtype in (torch.float32, torch.bfloat16) else None
    if code is None:
        x = x.float()
        code = 0
    if out is None:
        out = torch.empty(N_TENSOR_STATS + 1, dtype=torch.float32, device=x.device)
    ws = _workspace(x.device, int(_lib.lib().tdl_stats_workspace_bytes()))
    _lib.call("tdl_tensor_stats", ptr(x), code, x.numel(), ptr(out), ptr(ws), int(with_quantiles),
              stream_ptr(x.device))
    return out


def build_chunk_table(sizes: Sequence[int], device) -> torch.Tensor:
    """int64 table: C rows of (segment, start, end) followed by S+1 int32 'first chunk' offsets
    packed into int64 storage (read as int32 by the kernel)."""
    rows, first = [], []
    off = 0
    for s, n in enumerate(sizes):
        first.append(len(rows))
        st = off
        while st < off + n:
            en = min(st + CHUNK, off + n)
            rows.append((s, st, en))
            st = en
        if n == 0:
            pass
        off += n
    first.append(len(rows))
    C = len(rows)
    tab = torch.tensor([v for r in rows for v in r], dtype=torch.int64)
    f32 = np.array(first, dtype=np.int32)
    if f32.size % 2:
        f32 = np.concatenate([f32, np.zeros(1, np.int32)])
    tail = torch.from_numpy(f32.view(np.int64).copy())
    return torch.cat([tab, tail]).to(device), C


class FlatGradStats:
    """Segmented statistics over a stage's flat fp32 gradient (one segment per parameter).

    ``compute`` runs the whole pass.  The engine can instead run the per-chunk partial pass in
    pieces while the backward is still going (``partial(lo, hi)`` over chunk ranges, on the
    verifier's side stream, as each layer's gradient becomes final: ``chunk_range_of``), and then
    ``compute`` only adds the segment / summary / quantile stages."""

    def __init__(self, sizes: Sequence[int], device, ref_beta: float = 0.9, track_reference: bool = True):
        self.sizes = list(sizes)
        self.S = len(self.sizes)
        self.n = int(sum(self.sizes))
        self.device = torch.device(device)
        self.ref_beta = float(ref_beta)
        self.ref = torch.zeros(self.n, dtype=torch.float32, device=self.device) if track_reference else None
        self.ref_valid = False
        self.out = torch.zeros(18 + 2 * self.S, dtype=torch.float32, device=self.device)
        # chunk ranges per segment (CPU mirror of the device table): first[s] .. first[s+1]
        self.seg_first = [0]
        for n in self.sizes:
            self.seg_first.append(self.seg_first[-1] + (n + CHUNK - 1) // CHUNK)
        self._done = 0               # chunks whose partial already ran this step (prefix-free count)
        self._ranges: List[Tuple[int, int]] = []
        self.fused_segs = set()      # segments whose partial ran inside their weight-gradient reduce
        self._offs = [0]
        for n in self.sizes:
            self._offs.append(self._offs[-1] + n)
        if self.device.type == "cuda":
            self.table, self.C = build_chunk_table(self.sizes, self.device)
            nbytes = int(_lib.lib().tdl_grad_stats_ws_bytes(self.C, self.S)) + 64
            self.ws = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        else:
            self.C = self.seg_first[-1]

    def chunk_range_of(self, seg_lo: int, seg_hi: int) -> Tuple[int, int]:
        return self.seg_first[seg_lo], self.seg_first[seg_hi]

    def partial(self, flat_grad: torch.Tensor, c0: int, c1: int, stream=None) -> None:
        """Partial pass over chunks [c0, c1) (each chunk at most once per step)."""
        if not flat_grad.is_cuda or c1 <= c0:
            return
        _lib.call("tdl_grad_stats_partial", ptr(flat_grad), ptr(self.ref), ptr(self.table), self.C, self.S, c0, c1,
                  self.ref_beta, ptr(self.ws), int(self.ref_valid),
                  stream.cuda_stream if stream is not None else stream_ptr(flat_grad.device))
        self._ranges.append((c0, c1))
        self._done += c1 - c0

    def reduce_partial(self, flat_grad: torch.Tensor, seg: int, slabs: torch.Tensor, nsplit: int) -> bool:
        """Complete segment ``seg``'s gradient from split-K slabs ([nsplit][numel] fp32; the
        weight-gradient GEMM's partial products) AND run its chunks' partial pass in the same
        kernel, on the current stream: the final gradient is never re-read.  Bit-identical to
        ``tdl_splitk_reduce_add`` followed by ``partial``.  False when the segment's offset / size
        are not 16-byte multiples (the caller then reduces the plain way)."""
        off = sum(self.sizes[:seg]) if not hasattr(self, "_offs") else self._offs[seg]
        n = self.sizes[seg]
        c0, c1 = self.seg_first[seg], self.seg_first[seg + 1]
        if off % 4 or n % 4 or c1 <= c0 or not flat_grad.is_cuda:
            return False
        _lib.call("tdl_grad_stats_reduce_partial", ptr(flat_grad), ptr(slabs), int(nsplit), int(off), int(n),
                  ptr(self.ref), ptr(self.table), self.C, self.S, c0, c1, self.ref_beta, ptr(self.ws),
                  int(self.ref_valid), stream_ptr(flat_grad.device))
        self._ranges.append((c0, c1))
        self._done += c1 - c0
        self.fused_segs.add(seg)
        return True

    def compute(self, flat_grad: torch.Tensor, with_quantiles: bool = True) -> torch.Tensor:
        """Returns the device vector [18 + 2S]: GRAD_STATS(17), nonfinite, norms[S], cos[S]."""
        if flat_grad.is_cuda:
            dev = flat_grad.device
            if self._done == 0:
                _lib.call("tdl_grad_stats", ptr(flat_grad), ptr(self.ref), ptr(self.table), self.C, ptr(self.out),
                          self.n, self.ref_beta, self.S, ptr(self.ws), int(self.ref_valid), int(with_quantiles),
                          stream_ptr(dev))
            else:
                # the chunks no early partial covered (e.g. tied weights reduced after the backward)
                covered = sorted(self._ranges)
                pos = 0
                for lo, hi in covered + [(self.C, self.C)]:
                    if lo > pos:
                        self.partial(flat_grad, pos, lo)
                    pos = max(pos, hi)
                if self._done != self.C:
                    raise RuntimeError(f"grad stats: {self._done} chunk partials for {self.C} chunks")
                _lib.call("tdl_grad_stats_final", ptr(flat_grad), ptr(self.table), self.C, ptr(self.out), self.n,
                          self.S, ptr(self.ws), int(self.ref_valid), int(with_quantiles), stream_ptr(dev))
        else:
            self.out.copy_(self._cpu(flat_grad))
        self._done = 0
        self._ranges = []
        self.fused_segs = set()
        if self.ref is not None:
            self.ref_valid = True
        return self.out

    def _tracked_mask(self) -> torch.Tensor:
        """Elements whose EMA reference is kept (chunks c with c % REF_STRIDE == 0, as the kernel)."""
        m = getattr(self, "_tmask", None)
        if m is None:
            m = torch.zeros(self.n, dtype=torch.bool)
            off, c = 0, 0
            for n in self.sizes:
                st = off
                while st < off + n:
                    en = min(st + CHUNK, off + n)
                    if c % REF_STRIDE == 0:
                        m[st:en] = True
                    c += 1
                    st = en
                off += n
            self._tmask = m
        return m

    def _cpu(self, g: torch.Tensor) -> torch.Tensor:
        st = _cpu_stats(g)
        gf = g.detach().float()
        segs = torch.split(gf, self.sizes)
        norms = torch.stack([s.norm() for s in segs]) if segs else torch.zeros(0)
        tm = self._tracked_mask()
        if self.ref is not None and self.ref_valid:
            cos = []
            for a, r, t in zip(segs, torch.split(self.ref, self.sizes), torch.split(tm, self.sizes)):
                at, rt = a[t], r[t]
                den = float(at.norm() * rt.norm())
                cos.append(float((at * rt).sum()) / den if den > 0 else 2.0)
            cos = torch.tensor(cos)
        else:
            cos = torch.ones(self.S)
        if self.ref is not None:
            gg = torch.nan_to_num(gf, nan=0.0, posinf=0.0, neginf=0.0)
            if self.ref_valid:
                self.ref[tm] = self.ref[tm] * self.ref_beta + gg[tm] * (1 - self.ref_beta)
            else:
                self.ref[tm] = gg[tm]
        valid = cos <= 1.5
        cmean = float(cos[valid].mean()) if valid.any() else 1.0
        extra = torch.tensor([float(self.S), float(norms.mean()) if self.S else 0.0,
                              float(norms.std(unbiased=False)) if self.S else 0.0,
                              float(norms.max()) if self.S else 0.0, cmean if self.S else 1.0])
        return torch.cat([st[:12], extra, st[12:13], norms.float(), cos.float()])


class FlatSumSq:
    """Bare clipping norm for runs with verification off: sum_s w_s ||g_s||^2 over the flat
    gradient's segments (one read of the gradient, no moments / reference / quantiles)."""

    def __init__(self, sizes: Sequence[int], device):
        self.sizes = list(sizes)
        self.device = torch.device(device)
        self.out = torch.zeros(1, dtype=torch.float32, device=self.device)
        if self.device.type == "cuda" and self.sizes:
            self.table, self.C = build_chunk_table(self.sizes, self.device)
            self.ws = torch.empty(max(1, self.C), dtype=torch.float64, device=self.device)

    def compute(self, flat_grad: torch.Tensor, seg_w: torch.Tensor) -> torch.Tensor:
        if not self.sizes:
            self.out.zero_()
        elif flat_grad.is_cuda:
            _lib.call("tdl_grad_sumsq", ptr(flat_grad), ptr(self.table), self.C, ptr(seg_w), ptr(self.ws),
                      ptr(self.out), stream_ptr(flat_grad.device))
        else:
            segs = torch.split(flat_grad.detach().float(), self.sizes)
            sq = torch.stack([(x * x).sum() for x in segs])
            self.out.copy_((sq * seg_w[:len(self.sizes)].to(sq.device)).sum().reshape(1))
        return self.out


def grad_stats(grads: Sequence[torch.Tensor], reference: Optional[Sequence[torch.Tensor]] = None,
               cosine_mode: str = "reference") -> torch.Tensor:
    """GRAD_STATS vector [17] for an arbitrary list of (GPU) gradient tensors."""
    grads = [g.detach() for g in grads]
    dev = grads[0].device
    flat = torch.cat([g.float().reshape(-1) for g in grads])
    fs = FlatGradStats([g.numel() for g in grads], dev, track_reference=reference is not None)
    if reference is not None:
        fs.ref.copy_(torch.cat([r.float().reshape(-1) for r in reference]))
        fs.ref_valid = True
    out = fs.compute(flat)
    vec = out[:17].clone()
    if cosine_mode == "pairwise":
        from ..security.attack_detection import _cosine
        vec[16] = _cosine(grads, None, "pairwise")
    return vec


def _lower_upper_median(x: torch.Tensor) -> torch.Tensor:
    """Column medians with the kernel's convention (mean of the two middle values when even)."""
    s, _ = torch.sort(x, dim=0)
    n = s.shape[0]
    return s[n // 2] if n % 2 else 0.5 * (s[n // 2 - 1] + s[n // 2])


class DeviceZScore:
    """Device ring-buffer baseline + z-score decision for one monitored signal (K4)."""

    # csrc/stats.hip ZS_EARLY_MIN / ZS_EARLY_FACTOR.  3x: the clean ResNet-50 stages of attack config 4
    # reached |z| 12-17 right after a re-shard (profiles/r3_cfg_reshard.jsonl), gradient poisoning
    # reads 28-42
    EARLY_MIN, EARLY_FACTOR = 8, 3.0

    def __init__(self, k: int, device, history: int = 1000, warmup: int = 10, z_decision: float = 2.5,
                 exclude_current: bool = True, max_quarantine: int = 50, robust=True, window: int = 100,
                 rel_floor: float = 0.02, agg: str = "mean", abs_floor: float = 0.0, early_gate: bool = False):
        """``robust``: 1/True = median / 1.4826*MAD over the ``window`` most recent entries; 2 or
        "detrend" = the same about a robust linear trend of the window (the drift of learning:
        line through the medians of the window's recent and older halves), scale floored at
        ``rel_floor`` * |centre|; 0/False = the reference's mean / population std over the whole
        ``history``.  ``agg``: "mean" (the reference's rule: mean |z| over the features) or "max"
        (largest |z|: for short, targeted feature vectors)."""
        self.k, self.history, self.warmup = k, history, warmup
        # during warm-up, once EARLY_MIN entries exist, flag (and keep out of the baseline) gross
        # outliers above EARLY_FACTOR x z_decision (robust baselines only)
        self.early_gate = bool(early_gate)
        self.agg_max = agg == "max"
        self.robust = 2 if robust == "detrend" else int(robust)
        self.window = int(min(window, 128))
        self.rel_floor = float(rel_floor)
        self.abs_floor = float(abs_floor)
        self.z_decision = z_decision
        self.exclude_current = exclude_current
        self.max_quarantine = max_quarantine
        self.device = torch.device(device)
        self.ring = torch.zeros(history, k, dtype=torch.float32, device=self.device)
        self.state = torch.zeros(4, dtype=torch.int32, device=self.device)
        self.out = torch.zeros(4 + k, dtype=torch.float32, device=self.device)

    def rewarm(self, keep: Optional[int] = None) -> None:
        """Re-enter warm-up keeping only the ``keep`` (default EARLY_MIN) most recent baseline entries:
        the baseline refills from the new regime while the early gate still flags gross outliers
        (used after a re-plan: the training dynamics of a re-sharded pipeline shift)."""
        keep = self.EARLY_MIN if keep is None else int(keep)
        self.state[0:1].clamp_(max=keep)

    def observe(self, cur: torch.Tensor) -> torch.Tensor:
        """Returns device vector [4 + k]: flag, mean_z, confidence, n_valid, z[k] (-1 = skipped)."""
        cur = cur[: self.k].contiguous()
        if self.device.type == "cuda":
            _lib.call("tdl_zscore_detect", ptr(self.ring), ptr(self.state), ptr(cur), self.k, self.history,
                      self.warmup, self.z_decision, self.window, int(self.exclude_current), self.max_quarantine,
                      self.robust | (4 if self.agg_max else 0) | (8 if self.early_gate else 0), self.rel_floor,
                      self.abs_floor, ptr(self.out),
                      stream_ptr(self.device))
        else:
            self._cpu(cur)
        return self.out

    def _cpu(self, cur: torch.Tensor):
        count, head, qrun, seen = [int(v) for v in self.state.tolist()]
        H = self.history

        def append(c, h):
            self.ring[h] = cur
            return min(c + 1, H), (h + 1) % H

        if not self.exclude_current:
            count, head = append(count, head)
        ready = count >= self.warmup
        early = (not ready) and self.early_gate and bool(self.robust) and count >= self.EARLY_MIN
        zs = torch.full((self.k,), -1.0)
        if count > 0:
            if self.robust:
                wn = min(count, self.window)
                idx = [(head - 1 - j) % H for j in range(wn)]
                hist = self.ring[idx].clone()
                trend0 = torch.zeros(self.k)
                if self.robust == 2 and wn >= 8:
                    h = wn // 2
                    mr, mo = _lower_upper_median(hist[:h]), _lower_upper_median(hist[h:2 * h])
                    slope = (mr - mo) / h
                    tr = -1.0 - 0.5 * (h - 1)
                    tau = torch.tensor([-1.0 - j for j in range(wn)])[:, None]
                    hist = hist - (mr + slope * (tau - tr))
                    trend0 = mr + slope * (0.0 - tr)
                med = _lower_upper_median(hist)
                mean = trend0 + med
                sd = 1.4826 * _lower_upper_median((hist - med).abs())
                if self.robust == 2:
                    sd = torch.where(sd > 0, torch.maximum(sd, self.abs_floor + self.rel_floor * mean.abs()), sd)
            else:
                hist = self.ring[:count]
                mean = hist.mean(0)
                sd = hist.std(0, unbiased=False)
            for j in range(self.k):
                if (ready or early) and sd[j] > 0:
                    c = float(cur[j])
                    zs[j] = abs((c - float(mean[j])) / float(sd[j])) if math.isfinite(c) else 1e6
        valid = zs >= 0
        if self.agg_max:
            mz = float(zs[valid].max()) if valid.any() else 0.0
        else:
            mz = float(zs[valid].mean()) if valid.any() else 0.0
        flag = (mz > self.z_decision) if ready else (early and mz > self.EARLY_FACTOR * self.z_decision)
        if self.exclude_current:
            if flag and qrun < self.max_quarantine:
                qrun += 1
            else:
                qrun = 0
                count, head = append(count, head)
        self.state.copy_(torch.tensor([count, head, qrun, seen + 1], dtype=torch.int32))
        self.out.copy_(torch.cat([torch.tensor([1.0 if flag else 0.0, mz, min(1.0, mz / 5.0), float(valid.sum())]),
                                  zs]))


def trust_update(values: torch.Tensor, counts: torch.Tensor, status: torch.Tensor, metrics: torch.Tensor,
                 weights: torch.Tensor, threshold: float, decay_rate: float, dt: float = 1.0,
                 flags: Optional[torch.Tensor] = None, recovery: Optional[torch.Tensor] = None):
    """Fused trust update over all nodes (K5), in place on (values, counts, status)."""
    N = values.numel()
    if values.is_cuda:
        _lib.call("tdl_trust_update", ptr(values), ptr(counts), ptr(status), ptr(metrics.contiguous()),
                  ptr(weights), ptr(flags), ptr(recovery), N, float(threshold), float(decay_rate), float(dt),
                  stream_ptr(values.device))
        return
    from ..core.trust_manager import NodeStatus, STATUS_CODES, STATUS_FROM_CODE, next_status
    w = weights.double().tolist()
    for i in range(N):
        st = STATUS_FROM_CODE[int(status[i])]
        if st == NodeStatus.OFFLINE:
            continue
        old = float(values[i])
        if flags is not None and int(flags[i]):
            st, old = NodeStatus.COMPROMISED, 0.1
        m = metrics[i].double().tolist()
        comp = [1 - min(1.0, m[0]), m[1], 1 - min(1.0, m[2] / 10.0), min(1.0, m[3]), 1 - min(1.0, m[4]), m[5]]
        score = min(1.0, max(0.0, sum(a * b for a, b in zip(w, comp))))
        fin = 0.9 * old * math.exp(-decay_rate * dt) + 0.1 * score
        if st == NodeStatus.RECOVERING and recovery is not None:
            fin += float(recovery[i])
        fin = min(1.0, max(0.0, fin))
        values[i] = fin
        status[i] = STATUS_CODES[next_status(st, fin, threshold)]
        counts[i] += 1


def kl_div_softmax(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """KL(softmax(b) || softmax(a)) with 'batchmean' over the last dim (attack_detector.py:172-176)."""
    a2 = a.detach().float().reshape(-1, a.shape[-1]).contiguous()
    b2 = b.detach().float().reshape(-1, b.shape[-1]).contiguous()
    if a2.is_cuda:
        out = torch.empty(1, dtype=torch.float32, device=a2.device)
        _lib.call("tdl_kl_div_softmax", ptr(a2), ptr(b2), a2.shape[0], a2.shape[1], ptr(out), stream_ptr(a2.device))
        return out[0]
    return torch.nn.functional.kl_div(torch.log_softmax(a2, -1), torch.softmax(b2, -1), reduction="batchmean")


def cosine_gram(xs: List[torch.Tensor]) -> torch.Tensor:
    """N x N cosine similarity of flattened tensors (K6).  GPU: the native two-phase kernel reads
    the N tensors in place through a pointer table (no stacked copy; fp64 accumulation, fixed
    reduction order); CPU / unusual inputs: the torch reference."""
    n = len(xs)
    if n and all(x.is_cuda for x in xs) and n <= 16:
        flat = [x.detach().reshape(-1) for x in xs]
        D = flat[0].numel()
        dt = flat[0].dtype
        if dt in (torch.float32, torch.bfloat16) and all(f.numel() == D and f.dtype == dt and f.is_contiguous()
                                                          for f in flat):
            dev = flat[0].device
            out = torch.empty(n, n, dtype=torch.float32, device=dev)
            ws = _workspace(dev, int(_lib.lib().tdl_gram_ws_bytes()))
            table = (ctypes.c_void_p * n)(*[f.data_ptr() for f in flat])
            _lib.call("tdl_cosine_gram", ctypes.cast(table, ctypes.c_void_p), n, D, _lib.DTYPE_CODE[dt], ptr(out),
                      ptr(ws), stream_ptr(dev))
            return out
    X = torch.stack([x.detach().float().reshape(-1) for x in xs])
    nrm = X.norm(dim=1).clamp(min=1e-30)
    G = X @ X.t()
    return G / (nrm[:, None] * nrm[None, :])


_pos_w: Dict = {}


def _position_weights(n: int, device) -> torch.Tensor:
    key = (n, str(device))
    w = _pos_w.get(key)
    if w is None:
        if len(_pos_w) > 64:
            _pos_w.clear()
        w = _pos_w[key] = (torch.arange(n, dtype=torch.float64, device=device) % 1021) + 1
    return w


def checksum(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Deterministic (sum, sum of squares, position-weighted sum) of a flat buffer, float64 [3].
    Bit-identical data -> bit-identical result (fixed reduction order; csrc/stats.hip)."""
    x = x.reshape(-1)
    if out is None:
        out = torch.empty(3, dtype=torch.float64, device=x.device)
    if x.is_cuda and x.dtype == torch.bfloat16 and x.data_ptr() % 16 == 0:
        ws = torch.empty(3 * 2048, dtype=torch.float64, device=x.device)
        _lib.call("tdl_checksum_bf16", ptr(x), x.numel(), ptr(ws), ptr(out), stream_ptr(x.device))
        return out
    v = x.double()
    w = _position_weights(v.numel(), v.device)
    out.copy_(torch.stack([v.sum(), (v * v).sum(), (v * w).sum()]))
    return out
