"""Trust layer: per-node trust scores, status state machine and trust exports.

Behavioural parity target: reference ``trust_manager.py`` (TrustManager, NodeStatus,
TrustScore, NodeMetrics; trust_manager.py:18-398).  The public API and every numeric
default are kept, with these documented changes:

* ``decay_clock`` — the reference decays trust by *wall-clock* seconds between updates
  (trust_manager.py:112-114), which makes trust depend on step speed.  The
  default here is ``"step"``: the elapsed time is measured in training steps, so the
  same run always gives the same trust trajectory.  ``decay_clock="wall"`` restores the
  reference behaviour; an injectable ``clock`` makes it testable.
* ``mark_compromised`` records the trust value *before* the penalty (A14).
* ``recovery_rate`` is actually used: while a node is RECOVERING each update adds
  ``recovery_rate`` on top of the EMA (A15).
* ``calculate_system_trust`` guards the all-zero case (A17).
* ``decay_rate`` / ``recovery_rate`` constructor kwargs from the README facade
  (README.md:71-75, A20).

The same update is available as a fused device kernel over all nodes at once
(``trustworthy_dl.ops.trust_update``); ``TrustManager.ingest_device_update`` folds a
device-side result back into this host object without recomputing it.
"""
from __future__ import annotations

import json
import logging
import math
import time
from collections import defaultdict, deque
from dataclasses import dataclass, field, asdict
from enum import Enum
from typing import Callable, Dict, List, Optional

import numpy as np

logger = logging.getLogger(__name__)

# Order matters: it is the integer encoding used by the device kernel.
class NodeStatus(Enum):
    TRUSTED = "trusted"
    SUSPICIOUS = "suspicious"
    COMPROMISED = "compromised"
    RECOVERING = "recovering"
    OFFLINE = "offline"


STATUS_CODES = {s: i for i, s in enumerate(NodeStatus)}
STATUS_FROM_CODE = {i: s for s, i in STATUS_CODES.items()}

# Trust metric order used by the device kernel's [N, 6] metric matrix.
METRIC_NAMES = (
    "output_deviation",
    "gradient_consistency",
    "communication_latency",
    "resource_utilization",
    "error_rate",
    "uptime",
)

DEFAULT_TRUST_WEIGHTS = {
    "output_deviation": 0.3,
    "gradient_consistency": 0.3,
    "communication_latency": 0.1,
    "resource_utilization": 0.1,
    "error_rate": 0.15,
    "uptime": 0.05,
}

EMA_ALPHA = 0.1          # trust_manager.py:117
COMPROMISED_BELOW = 0.3  # trust_manager.py:166
RECOVERING_ABOVE = 0.8   # trust_manager.py:170
RECOVERED_ABOVE = 0.9    # trust_manager.py:172
COMPROMISE_PENALTY = 0.1 # trust_manager.py:186


@dataclass
class TrustScore:
    """Trust value with bookkeeping (reference trust_manager.py:25-32)."""
    value: float
    last_updated: float
    update_count: int
    decay_rate: float = 0.01
    recovery_rate: float = 0.005


@dataclass
class NodeMetrics:
    """Raw per-node behaviour metrics (reference trust_manager.py:34-42)."""
    output_deviation: float = 0.0
    gradient_consistency: float = 1.0
    communication_latency: float = 0.0
    resource_utilization: float = 0.0
    error_rate: float = 0.0
    uptime: float = 1.0

    def as_vector(self) -> List[float]:
        return [float(getattr(self, k)) for k in METRIC_NAMES]


def trust_components(m: NodeMetrics) -> Dict[str, float]:
    """Map raw metrics to [0,1] "higher is better" components (trust_manager.py:145-152)."""
    return {
        "output_deviation": 1.0 - min(1.0, m.output_deviation),
        "gradient_consistency": m.gradient_consistency,
        "communication_latency": 1.0 - min(1.0, m.communication_latency / 10.0),
        "resource_utilization": min(1.0, m.resource_utilization),
        "error_rate": 1.0 - min(1.0, m.error_rate),
        "uptime": m.uptime,
    }


def next_status(current: NodeStatus, score: float, threshold: float) -> NodeStatus:
    """Status transition table (trust_manager.py:162-181), shared with the device kernel."""
    if score < COMPROMISED_BELOW:
        return NodeStatus.COMPROMISED
    if score < threshold:
        return NodeStatus.SUSPICIOUS
    if current == NodeStatus.COMPROMISED and score > RECOVERING_ABOVE:
        return NodeStatus.RECOVERING
    if current == NodeStatus.RECOVERING and score > RECOVERED_ABOVE:
        return NodeStatus.TRUSTED
    if score >= threshold:
        return NodeStatus.TRUSTED
    return current


class TrustManager:
    """Dynamic trust scoring and node status management.

    ``TrustManager(num_nodes, trust_threshold=0.7, initial_trust=1.0, max_history=1000)``
    matches reference trust_manager.py:49-50.  ``num_nodes`` may be omitted (README facade,
    README.md:71-75); it is then bound by ``DistributedTrainer`` via :meth:`resize`.
    """

    def __init__(self, num_nodes: int = 0, trust_threshold: float = 0.7,
                 initial_trust: float = 1.0, max_history: int = 1000,
                 decay_rate: float = 0.01, recovery_rate: float = 0.005,
                 decay_clock: str = "step", clock: Optional[Callable[[], float]] = None,
                 trust_weights: Optional[Dict[str, float]] = None):
        if decay_clock not in ("step", "wall"):
            raise ValueError(f"decay_clock must be 'step' or 'wall', got {decay_clock!r}")
        self.num_nodes = int(num_nodes)
        self.trust_threshold = float(trust_threshold)
        self.default_threshold = float(trust_threshold)
        self.initial_trust = float(initial_trust)
        self.max_history = int(max_history)
        self.decay_rate = float(decay_rate)
        self.recovery_rate = float(recovery_rate)
        self.decay_clock = decay_clock
        self._clock = clock or time.time
        self._step = 0

        self.trust_scores: Dict[int, TrustScore] = {}
        self.node_status: Dict[int, NodeStatus] = {}
        self.node_metrics: Dict[int, NodeMetrics] = {}
        self._last_step: Dict[int, int] = {}

        self.trust_history: Dict[int, deque] = defaultdict(lambda: deque(maxlen=self.max_history))
        self.attack_history: Dict[int, List] = defaultdict(list)
        self.performance_history: Dict[int, deque] = defaultdict(lambda: deque(maxlen=self.max_history))

        self.trust_weights = dict(trust_weights or DEFAULT_TRUST_WEIGHTS)
        for node_id in range(self.num_nodes):
            self.initialize_node(node_id)
        logger.info("TrustManager initialized for %d nodes", self.num_nodes)

    # ------------------------------------------------------------------ clock
    def now(self) -> float:
        return float(self._clock())

    def advance_step(self, step: Optional[int] = None) -> int:
        """Advance the logical clock used by ``decay_clock="step"``."""
        self._step = self._step + 1 if step is None else int(step)
        return self._step

    @property
    def current_step(self) -> int:
        return self._step

    def resize(self, num_nodes: int):
        """Bind / grow the node set (README facade constructs without num_nodes)."""
        for node_id in range(self.num_nodes, num_nodes):
            self.initialize_node(node_id)
        self.num_nodes = max(self.num_nodes, int(num_nodes))

    # ------------------------------------------------------------------ core
    def initialize_node(self, node_id: int):
        self.trust_scores[node_id] = TrustScore(
            value=self.initial_trust, last_updated=self.now(), update_count=0,
            decay_rate=self.decay_rate, recovery_rate=self.recovery_rate)
        self.node_status[node_id] = NodeStatus.TRUSTED
        self.node_metrics[node_id] = NodeMetrics()
        self._last_step[node_id] = self._step

    def _elapsed(self, node_id: int) -> float:
        if self.decay_clock == "wall":
            return self.now() - self.trust_scores[node_id].last_updated
        return float(max(1, self._step - self._last_step.get(node_id, self._step - 1)))

    def update_trust_score(self, node_id: int, output_deviation: float,
                           gradient_consistency: float, **kwargs):
        """EMA trust update with temporal decay (trust_manager.py:92-140)."""
        if node_id not in self.trust_scores:
            self.initialize_node(node_id)
            self.num_nodes = max(self.num_nodes, node_id + 1)
        metrics = self.node_metrics[node_id]
        metrics.output_deviation = float(output_deviation)
        metrics.gradient_consistency = float(gradient_consistency)
        for key, value in kwargs.items():
            if hasattr(metrics, key):
                setattr(metrics, key, float(value))

        new_trust = self._calculate_trust_score(node_id, metrics)
        old = self.trust_scores[node_id]
        decay = math.exp(-old.decay_rate * self._elapsed(node_id))
        final = (1.0 - EMA_ALPHA) * old.value * decay + EMA_ALPHA * new_trust
        if self.node_status[node_id] == NodeStatus.RECOVERING:
            final += old.recovery_rate
        final = float(min(1.0, max(0.0, final)))

        stamp = self.now()
        self.trust_scores[node_id] = TrustScore(
            value=final, last_updated=stamp, update_count=old.update_count + 1,
            decay_rate=old.decay_rate, recovery_rate=old.recovery_rate)
        self._last_step[node_id] = self._step
        self._update_node_status(node_id, final)
        self.trust_history[node_id].append({
            "timestamp": stamp, "step": self._step, "trust_score": final,
            "metrics": asdict(metrics)})
        return final

    def _calculate_trust_score(self, node_id: int, metrics: NodeMetrics) -> float:
        comps = trust_components(metrics)
        score = sum(self.trust_weights[k] * v for k, v in comps.items())
        return float(min(1.0, max(0.0, score)))

    def _update_node_status(self, node_id: int, trust_score: float):
        cur = self.node_status[node_id]
        new = next_status(cur, trust_score, self.trust_threshold)
        if new != cur:
            logger.info("Node %d status changed: %s -> %s", node_id, cur.value, new.value)
            self.node_status[node_id] = new

    def ingest_device_update(self, values, statuses, metrics=None, update_counts=None):
        """Adopt the result of the fused device trust kernel for all nodes.

        ``values``/``statuses`` are host sequences of length ``num_nodes`` (status as int
        codes, see ``STATUS_CODES``); ``metrics`` an optional [N, 6] host array.
        """
        stamp = self.now()
        for nid in range(len(values)):
            old = self.trust_scores.get(nid)
            if old is None:
                self.initialize_node(nid)
                old = self.trust_scores[nid]
            cnt = int(update_counts[nid]) if update_counts is not None else old.update_count + 1
            self.trust_scores[nid] = TrustScore(float(values[nid]), stamp, cnt,
                                                old.decay_rate, old.recovery_rate)
            new_status = STATUS_FROM_CODE[int(statuses[nid])]
            if new_status != self.node_status.get(nid):
                logger.info("Node %d status changed: %s -> %s", nid,
                            self.node_status.get(nid, NodeStatus.OFFLINE).value, new_status.value)
            self.node_status[nid] = new_status
            self._last_step[nid] = self._step
            if metrics is not None:
                m = self.node_metrics[nid]
                for k, v in zip(METRIC_NAMES, metrics[nid]):
                    setattr(m, k, float(v))
            self.trust_history[nid].append({
                "timestamp": stamp, "step": self._step, "trust_score": float(values[nid]),
                "metrics": asdict(self.node_metrics[nid])})

    # ------------------------------------------------------------------ events
    def mark_compromised(self, node_id: int, attack_type: str = "unknown"):
        """Hard penalty after a detection (trust_manager.py:183-196; A14 fixed)."""
        if node_id not in self.trust_scores:
            self.initialize_node(node_id)
        previous = self.trust_scores[node_id].value
        self.node_status[node_id] = NodeStatus.COMPROMISED
        self.trust_scores[node_id].value = COMPROMISE_PENALTY
        self.attack_history[node_id].append({
            "timestamp": self.now(), "step": self._step, "attack_type": attack_type,
            "previous_trust": previous})
        logger.warning("Node %d marked as compromised: %s", node_id, attack_type)

    def mark_offline(self, node_id: int, reason: str = "heartbeat timeout"):
        """OFFLINE is set by the runtime's heartbeat / collective timeout watchdog."""
        self.node_status[node_id] = NodeStatus.OFFLINE
        self.node_metrics.setdefault(node_id, NodeMetrics()).uptime = 0.0
        logger.warning("Node %d marked offline: %s", node_id, reason)

    def initiate_recovery(self, node_id: int):
        """COMPROMISED -> RECOVERING with a boosted recovery rate (trust_manager.py:198-206)."""
        if self.node_status.get(node_id) == NodeStatus.COMPROMISED:
            self.node_status[node_id] = NodeStatus.RECOVERING
            self.trust_scores[node_id].recovery_rate = 0.02
            logger.info("Recovery initiated for node %d", node_id)

    # ------------------------------------------------------------------ queries
    def get_trust_score(self, node_id: int) -> float:
        s = self.trust_scores.get(node_id)
        return 0.0 if s is None else float(s.value)

    def get_node_status(self, node_id: int) -> NodeStatus:
        return self.node_status.get(node_id, NodeStatus.OFFLINE)

    def _nodes_with(self, status: NodeStatus) -> List[int]:
        return [n for n in range(self.num_nodes) if self.node_status.get(n) == status]

    def get_trusted_nodes(self) -> List[int]:
        return self._nodes_with(NodeStatus.TRUSTED)

    def get_suspicious_nodes(self) -> List[int]:
        return self._nodes_with(NodeStatus.SUSPICIOUS)

    def get_compromised_nodes(self) -> List[int]:
        return self._nodes_with(NodeStatus.COMPROMISED)

    def can_assign_task(self, node_id: int) -> bool:
        return self.node_status.get(node_id, NodeStatus.OFFLINE) in (
            NodeStatus.TRUSTED, NodeStatus.RECOVERING)

    def select_best_nodes(self, num_nodes: int, distance: Optional[Callable[[int], float]] = None) -> List[int]:
        """Top-k assignable nodes by trust; optional tie-break by a distance function
        (e.g. xGMI hop distance to a reference GPU)."""
        cands = [n for n in range(self.num_nodes) if self.can_assign_task(n)]
        if distance is None:
            cands.sort(key=lambda n: -self.get_trust_score(n))
        else:
            cands.sort(key=lambda n: (-self.get_trust_score(n), distance(n)))
        return cands[:num_nodes]

    def calculate_system_trust(self) -> float:
        """Trust-weighted mean of trust values (trust_manager.py:259-270; A17 guarded)."""
        vals = np.array([s.value for s in self.trust_scores.values()], dtype=np.float64)
        if vals.size == 0 or vals.sum() <= 0.0:
            return 0.0
        return float(np.average(vals, weights=vals))

    def get_trust_statistics(self) -> Dict:
        vals = [s.value for s in self.trust_scores.values()]
        if not vals:
            return {}
        return {
            "mean_trust": float(np.mean(vals)),
            "std_trust": float(np.std(vals)),
            "min_trust": float(np.min(vals)),
            "max_trust": float(np.max(vals)),
            "system_trust": self.calculate_system_trust(),
            "node_status_counts": {
                st.value: sum(1 for s in self.node_status.values() if s == st) for st in NodeStatus},
            "total_attacks": sum(len(a) for a in self.attack_history.values()),
        }

    def get_node_history(self, node_id: int, limit: int = 100) -> List[Dict]:
        if node_id not in self.trust_history:
            return []
        hist = list(self.trust_history[node_id])
        return hist[-limit:] if limit else hist

    def export_trust_data(self, filepath: str):
        """JSON export with the reference schema (trust_manager.py:302-331)."""
        data = {
            "trust_scores": {str(n): {"value": s.value, "last_updated": s.last_updated,
                                      "update_count": s.update_count}
                             for n, s in self.trust_scores.items()},
            "node_status": {str(n): st.value for n, st in self.node_status.items()},
            "trust_history": {str(n): list(h) for n, h in self.trust_history.items()},
            "attack_history": {str(n): a for n, a in self.attack_history.items()},
            "statistics": self.get_trust_statistics(),
        }
        with open(filepath, "w") as f:
            json.dump(data, f, indent=2, default=float)
        logger.info("Trust data exported to %s", filepath)

    def adaptive_threshold_adjustment(self) -> float:
        """Threshold adaptation (trust_manager.py:333-348); called once per epoch by the trainer."""
        mean_trust = self.get_trust_statistics().get("mean_trust", 0.7)
        if mean_trust < 0.5:
            self.trust_threshold = max(0.3, mean_trust - 0.1)
        elif mean_trust > 0.9:
            self.trust_threshold = min(0.8, mean_trust - 0.1)
        else:
            self.trust_threshold += 0.01 * (0.7 - self.trust_threshold)
        return self.trust_threshold

    def predict_node_reliability(self, node_id: int, horizon: int = 10) -> float:
        """Linear trend extrapolation over the last 10 scores (trust_manager.py:350-368)."""
        hist = self.trust_history.get(node_id)
        if hist is None or len(hist) < 5:
            return self.get_trust_score(node_id)
        recent = [e["trust_score"] for e in list(hist)[-10:]]
        x = np.arange(len(recent))
        slope, icpt = np.polyfit(x, recent, 1)
        return float(np.clip(slope * (len(recent) + horizon) + icpt, 0.0, 1.0))

    def get_recommendations(self) -> List[str]:
        recs = []
        stats = self.get_trust_statistics()
        if stats.get("mean_trust", 1.0) < 0.6:
            recs.append("System trust is low - consider investigating compromised nodes")
        if len(self.get_compromised_nodes()) > self.num_nodes * 0.3:
            recs.append("High number of compromised nodes - check security measures")
        if stats.get("total_attacks", 0) > 10:
            recs.append("Frequent attacks detected - strengthen attack detection")
        sus = self.get_suspicious_nodes()
        if sus:
            recs.append(f"Monitor suspicious nodes: {sus}")
        return recs

    def reset_node_trust(self, node_id: int):
        self.initialize_node(node_id)
        logger.info("Trust reset for node %d", node_id)

    # ------------------------------------------------------------------ state
    def state_dict(self) -> Dict:
        return {
            "num_nodes": self.num_nodes, "trust_threshold": self.trust_threshold,
            "step": self._step,
            "scores": {n: asdict(s) for n, s in self.trust_scores.items()},
            "status": {n: s.value for n, s in self.node_status.items()},
            "metrics": {n: asdict(m) for n, m in self.node_metrics.items()},
            "attack_history": {n: list(a) for n, a in self.attack_history.items()},
            "last_step": dict(self._last_step),
        }

    def load_state_dict(self, sd: Dict):
        self.num_nodes = int(sd["num_nodes"])
        self.trust_threshold = float(sd["trust_threshold"])
        self._step = int(sd["step"])
        self.trust_scores = {int(n): TrustScore(**s) for n, s in sd["scores"].items()}
        self.node_status = {int(n): NodeStatus(s) for n, s in sd["status"].items()}
        self.node_metrics = {int(n): NodeMetrics(**m) for n, m in sd["metrics"].items()}
        self.attack_history = defaultdict(list, {int(n): list(a) for n, a in sd["attack_history"].items()})
        self._last_step = {int(n): int(s) for n, s in sd["last_step"].items()}

    def weights_vector(self) -> List[float]:
        return [self.trust_weights[k] for k in METRIC_NAMES]

    def cleanup(self):
        logger.info("TrustManager cleanup completed")
