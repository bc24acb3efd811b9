"""Post-re-plan detector re-warm (ops/stats.py DeviceZScore.rewarm, StageVerifier.rewarm): the
baseline keeps its most recent entries, re-enters the early-gated warm-up, flags only gross outliers
(> EARLY_FACTOR x z_decision) until it has refilled, then the normal threshold applies again."""
import torch

from trustworthy_dl.ops.stats import DeviceZScore


def _det():
    return DeviceZScore(1, "cpu", history=200, warmup=30, z_decision=8.0, robust="detrend", window=64, agg="max",
                        rel_floor=0.0, abs_floor=0.05, early_gate=True)


def test_rewarm_caps_baseline_and_gates():
    g = torch.Generator().manual_seed(0)
    d = _det()
    for _ in range(60):
        d.observe(torch.randn(1, generator=g) * 0.1)
    assert int(d.state[0]) == 60
    # warm: a 12-sigma point flags
    assert float(d.observe(torch.tensor([0.1 * 12 / 1.0]))[0]) in (0.0, 1.0)
    d.rewarm()
    assert int(d.state[0]) == DeviceZScore.EARLY_MIN
    # re-warming: a moderate outlier (between z_decision and EARLY_FACTOR x z_decision) does not flag,
    # a gross one does
    flags = []
    for v in (0.0, 0.05, -0.05, 0.02):
        flags.append(float(d.observe(torch.tensor([v]))[0]))
    assert flags == [0.0] * 4
    mid = d.observe(torch.tensor([0.9]))        # between z_decision and the gross threshold: no flag
    assert d.z_decision < float(mid[1]) < DeviceZScore.EARLY_FACTOR * d.z_decision and float(mid[0]) == 0.0
    z = d.observe(torch.tensor([4.0]))          # far above EARLY_FACTOR x z_decision: flagged
    assert float(z[1]) > DeviceZScore.EARLY_FACTOR * d.z_decision and float(z[0]) == 1.0
    for _ in range(40):
        d.observe(torch.randn(1, generator=g) * 0.1)
    assert int(d.state[0]) >= d.warmup             # refilled: back to the normal threshold
