"""TrustManager math vs the reference formulas (trust_manager.py:92-368), injectable clock."""
import json
import math

import pytest

from trustworthy_dl.core.trust_manager import NodeStatus, TrustManager, next_status


class Clock:
    def __init__(self):
        self.t = 1000.0

    def __call__(self):
        return self.t


def ref_update(old, m, decay_rate=0.01, dt=1.0):
    comps = [1 - min(1, m[0]), m[1], 1 - min(1, m[2] / 10), min(1, m[3]), 1 - min(1, m[4]), m[5]]
    w = [0.3, 0.3, 0.1, 0.1, 0.15, 0.05]
    new = min(1.0, max(0.0, sum(a * b for a, b in zip(w, comps))))
    return min(1.0, max(0.0, 0.9 * old * math.exp(-decay_rate * dt) + 0.1 * new))


def test_defaults_and_init():
    tm = TrustManager(4)
    assert tm.trust_threshold == 0.7 and tm.initial_trust == 1.0 and tm.max_history == 1000
    assert all(tm.get_trust_score(i) == 1.0 for i in range(4))
    assert tm.get_trusted_nodes() == [0, 1, 2, 3]
    assert tm.get_node_status(99) == NodeStatus.OFFLINE
    assert tm.get_trust_score(99) == 0.0


def test_step_decay_matches_reference_formula():
    tm = TrustManager(1, decay_clock="step")
    v = 1.0
    for s in range(30):
        tm.advance_step()
        m = (0.1, 0.9, 0.5, 0.8, 0.0, 1.0)
        got = tm.update_trust_score(0, m[0], m[1], communication_latency=m[2], resource_utilization=m[3],
                                    error_rate=m[4], uptime=m[5])
        v = ref_update(v, m)
        assert abs(got - v) < 1e-12


def test_wall_clock_decay_compat():
    clk = Clock()
    tm = TrustManager(1, decay_clock="wall", clock=clk)
    clk.t += 5.0
    got = tm.update_trust_score(0, 0.0, 1.0)
    assert abs(got - ref_update(1.0, (0, 1, 0, 0, 0, 1), dt=5.0)) < 1e-12


def test_healthy_steady_state_and_worst():
    tm = TrustManager(2, decay_clock="wall", clock=Clock())  # dt = 0 -> reference steady state
    for _ in range(200):
        tm.update_trust_score(0, 0.0, 1.0)
        tm.update_trust_score(1, 1.0, 0.0)
    assert abs(tm.get_trust_score(0) - 0.9) < 1e-3       # SURVEY: 0.900 with util = 0
    assert abs(tm.get_trust_score(1) - 0.3) < 0.02       # ~0.31 worst metrics
    assert tm.get_node_status(1) in (NodeStatus.SUSPICIOUS, NodeStatus.COMPROMISED)


def test_status_machine():
    assert next_status(NodeStatus.TRUSTED, 0.29, 0.7) == NodeStatus.COMPROMISED
    assert next_status(NodeStatus.TRUSTED, 0.5, 0.7) == NodeStatus.SUSPICIOUS
    assert next_status(NodeStatus.COMPROMISED, 0.85, 0.7) == NodeStatus.RECOVERING
    assert next_status(NodeStatus.RECOVERING, 0.95, 0.7) == NodeStatus.TRUSTED
    assert next_status(NodeStatus.RECOVERING, 0.75, 0.7) == NodeStatus.TRUSTED
    assert next_status(NodeStatus.SUSPICIOUS, 0.7, 0.7) == NodeStatus.TRUSTED


def test_mark_compromised_records_previous_trust_and_recovers():
    tm = TrustManager(3, decay_clock="wall", clock=Clock())
    tm.mark_compromised(1, "gradient_poisoning")
    assert tm.get_trust_score(1) == pytest.approx(0.1)
    assert tm.attack_history[1][0]["previous_trust"] == 1.0   # A14 fixed
    assert tm.get_compromised_nodes() == [1]
    assert not tm.can_assign_task(1)
    n = 0
    while tm.get_node_status(1) != NodeStatus.TRUSTED and n < 100:
        tm.update_trust_score(1, 0.0, 1.0)
        n += 1
    assert n == 14  # SURVEY: 14 updates from mark_compromised back to TRUSTED


def test_recovery_rate_used():
    tm = TrustManager(1, decay_clock="wall", clock=Clock())
    tm.mark_compromised(0)
    tm.initiate_recovery(0)
    assert tm.get_node_status(0) == NodeStatus.RECOVERING
    v = tm.update_trust_score(0, 0.0, 1.0)
    assert v == pytest.approx(0.9 * 0.1 + 0.1 * 0.9 + 0.02)


def test_selection_system_trust_and_guard():
    tm = TrustManager(4)
    tm.trust_scores[0].value = 0.5
    tm.trust_scores[1].value = 0.9
    tm.node_status[2] = NodeStatus.COMPROMISED
    assert tm.select_best_nodes(2) == [3, 1]
    for s in tm.trust_scores.values():
        s.value = 0.0
    assert tm.calculate_system_trust() == 0.0  # A17: no ZeroDivisionError


def test_adaptive_threshold_predict_recommend(tmp_path):
    tm = TrustManager(3, decay_clock="wall", clock=Clock())
    for s in tm.trust_scores.values():
        s.value = 0.4
    assert tm.adaptive_threshold_adjustment() == pytest.approx(0.3)
    tm2 = TrustManager(1, decay_clock="wall", clock=Clock())
    for _ in range(10):
        tm2.update_trust_score(0, 1.0, 0.0)
    pred = tm2.predict_node_reliability(0)
    assert 0.0 <= pred <= tm2.get_trust_score(0)
    tm.mark_compromised(0)
    recs = tm.get_recommendations()
    assert any("low" in r for r in recs)
    p = tmp_path / "trust.json"
    tm.export_trust_data(str(p))
    d = json.loads(p.read_text())
    assert set(d) == {"trust_scores", "node_status", "trust_history", "attack_history", "statistics"}
    assert d["node_status"]["0"] == "compromised"


def test_state_dict_roundtrip():
    tm = TrustManager(3)
    tm.advance_step()
    tm.update_trust_score(0, 0.5, 0.5)
    tm.mark_compromised(2)
    tm2 = TrustManager(3)
    tm2.load_state_dict(tm.state_dict())
    assert tm2.get_trust_score(0) == tm.get_trust_score(0)
    assert tm2.get_node_status(2) == NodeStatus.COMPROMISED
