"""Per-node behaviour baselines feeding the trust metrics.

The reference imports ``NodeMonitor`` (distributed_trainer.py:20, 80) and queries
``get_expected_mean`` / ``get_expected_std`` (distributed_trainer.py:234-235) and
``get_expected_gradient_norms`` (distributed_trainer.py:259), but never ships the module
nor feeds it, so its baselines are always empty.  This implementation keeps
running EMA baselines fed by the trainer every step from the device statistic vectors,
plus the runtime signals behind the remaining trust metrics (trust_manager.py:38-42):
communication latency, resource utilisation, error rate and uptime (heartbeats).
"""
from __future__ import annotations

import time
from collections import defaultdict
from typing import Dict, List, Optional, Sequence

import numpy as np


class _EMA:
    __slots__ = ("value", "count", "beta")

    def __init__(self, beta: float):
        self.value = None
        self.count = 0
        self.beta = beta

    def update(self, x):
        x = np.asarray(x, dtype=np.float64)
        if self.value is None or np.shape(self.value) != np.shape(x):
            self.value = x.copy()
        else:
            self.value = self.beta * self.value + (1.0 - self.beta) * x
        self.count += 1
        return self.value


class NodeMonitor:
    """Running baselines per node (EMA, ``beta``) with a warm-up before they are reported."""

    def __init__(self, beta: float = 0.95, warmup: int = 5, heartbeat_timeout: float = 60.0):
        self.beta = beta
        self.warmup = warmup
        self.heartbeat_timeout = heartbeat_timeout
        self._out_mean: Dict[int, _EMA] = defaultdict(lambda: _EMA(self.beta))
        self._out_std: Dict[int, _EMA] = defaultdict(lambda: _EMA(self.beta))
        self._grad_norms: Dict[int, _EMA] = defaultdict(lambda: _EMA(self.beta))
        self.latency: Dict[int, float] = defaultdict(float)
        self.utilization: Dict[int, float] = defaultdict(float)
        self.error_rate: Dict[int, float] = defaultdict(float)
        self._errors: Dict[int, int] = defaultdict(int)
        self._observations: Dict[int, int] = defaultdict(int)
        self._last_heartbeat: Dict[int, float] = {}
        self._started = time.time()

    # ---------------------------------------------------------------- feeding
    def record_output(self, node_id: int, mean: float, std: float):
        self._out_mean[node_id].update(mean)
        self._out_std[node_id].update(std)

    def record_gradient_norms(self, node_id: int, norms: Sequence[float]):
        self._grad_norms[node_id].update(list(norms))

    def record_step(self, node_id: int, latency_s: float = 0.0, utilization: float = 0.0,
                    had_error: bool = False):
        self.latency[node_id] = float(latency_s)
        self.utilization[node_id] = float(utilization)
        self._observations[node_id] += 1
        self._errors[node_id] += int(bool(had_error))
        self.error_rate[node_id] = self._errors[node_id] / self._observations[node_id]
        self.heartbeat(node_id)

    def heartbeat(self, node_id: int, t: Optional[float] = None):
        self._last_heartbeat[node_id] = time.time() if t is None else t

    # ---------------------------------------------------------------- queries (reference API)
    def get_expected_mean(self, node_id: int) -> Optional[float]:
        e = self._out_mean.get(node_id)
        return None if e is None or e.count < self.warmup else float(e.value)

    def get_expected_std(self, node_id: int) -> Optional[float]:
        e = self._out_std.get(node_id)
        return None if e is None or e.count < self.warmup else float(e.value)

    def get_expected_gradient_norms(self, node_id: int) -> List[float]:
        e = self._grad_norms.get(node_id)
        return [] if e is None or e.count < self.warmup else [float(v) for v in e.value]

    def uptime(self, node_id: int, now: Optional[float] = None) -> float:
        now = time.time() if now is None else now
        last = self._last_heartbeat.get(node_id)
        if last is None:
            return 1.0
        return 0.0 if now - last > self.heartbeat_timeout else 1.0

    def is_alive(self, node_id: int, now: Optional[float] = None) -> bool:
        return self.uptime(node_id, now) > 0.0

    def runtime_metrics(self, node_id: int) -> Dict[str, float]:
        return {"communication_latency": self.latency[node_id],
                "resource_utilization": self.utilization[node_id],
                "error_rate": self.error_rate[node_id],
                "uptime": self.uptime(node_id)}

    def reset(self, node_id: int):
        for d in (self._out_mean, self._out_std, self._grad_norms):
            d.pop(node_id, None)


def output_deviation(mean: float, std: float, exp_mean: Optional[float], exp_std: Optional[float]) -> float:
    """Reference formula (distributed_trainer.py:228-248)."""
    if exp_mean is None or exp_std is None or exp_std <= 0:
        return 0.0
    return float(min(1.0, (abs(mean - exp_mean) / exp_std + abs(std - exp_std) / exp_std) / 2.0))


def gradient_consistency(norms: Sequence[float], expected: Sequence[float], symmetric: bool = True) -> float:
    """Per-tensor norm ratio score (distributed_trainer.py:250-271).

    ``symmetric=True`` penalises inflated norms too (min(r, 1/r)); the reference only
    penalises shrunken ones (min(1, r)), so a x10 poisoned gradient scored 1.0.
    """
    if len(norms) == 0:
        return 0.0
    if len(expected) == 0:
        return 1.0
    scores = []
    for n, e in zip(norms, expected):
        if e > 0:
            r = n / e
            scores.append(min(r, 1.0 / r) if (symmetric and r > 0) else min(1.0, r))
    return float(np.mean(scores)) if scores else 1.0
