"""AttackDetector decision logic vs reference semantics (attack_detector.py:71-363) and the F1 protocol
of BASELINE.md (100 clean steps, then 200 steps with p(attack)=0.2 on 4x[256,256] N(0,0.01) grads)."""
import numpy as np
import pytest
import torch

from trustworthy_dl.security.attack_detection import (AttackDetector, AttackType, GRAD_STATS, TENSOR_STATS,
                                                      numpy_tensor_statistics)


def test_numpy_stats_match_scipy():
    from scipy import stats
    x = np.random.default_rng(0).standard_normal(10000) * 3 + 1
    s = numpy_tensor_statistics(x)
    assert s["skewness"] == pytest.approx(float(stats.skew(x)), rel=1e-9)
    assert s["kurtosis"] == pytest.approx(float(stats.kurtosis(x)), rel=1e-9)
    assert s["std"] == pytest.approx(float(np.std(x)))
    assert s["percentile_25"] == pytest.approx(float(np.percentile(x, 25)))
    assert s["norm_l2"] == pytest.approx(float(np.linalg.norm(x)))


def test_output_anomaly_warmup_and_detection():
    det = AttackDetector()
    g = torch.Generator().manual_seed(0)
    for s in range(20):
        assert not det.detect_output_anomaly(torch.randn(4, 16, 64, generator=g), 0, s)
    assert det.detect_output_anomaly(torch.randn(4, 16, 64, generator=g) * 1.5 + 1.0, 0, 20)
    clean = sum(det.detect_output_anomaly(torch.randn(4, 16, 64, generator=g), 0, s) for s in range(21, 51))
    assert clean == 0


def test_classification_rules():
    ev = {"norm_l2": {"z_score": 6.0}}
    assert AttackDetector._classify_attack_type(ev, {}) == AttackType.GRADIENT_POISONING
    assert AttackDetector._classify_attack_type({"std": {"z_score": 4.5}}, {}) == AttackType.DATA_POISONING
    assert AttackDetector._classify_attack_type({"kurtosis": {"z_score": 3.5}}, {}) == AttackType.ADVERSARIAL_INPUT
    assert AttackDetector._classify_attack_type({"max": {"z_score": 3.5}}, {}) == AttackType.BYZANTINE
    assert AttackDetector._classify_attack_type({}, {}) is None


def test_mixed_shape_gradients_do_not_crash():
    det = AttackDetector(compat=True)  # reference pairwise cosine mode, restricted to equal shapes (A10)
    grads = [torch.randn(8, 4), torch.randn(3), torch.randn(8, 4)]
    for s in range(12):
        det.detect_gradient_poisoning(grads, 0, s)


def _f1_run(det, transform, seed=0, warm=100, steps=200, p=0.2):
    rng = np.random.default_rng(seed)
    tp = fp = fn = 0
    for s in range(warm + steps):
        grads = [torch.from_numpy(rng.normal(0, 0.01, (256, 256)).astype(np.float32)) for _ in range(4)]
        attack = s >= warm and rng.random() < p
        if attack:
            grads = [transform(g) for g in grads]
        flagged = det.detect_gradient_poisoning(grads, 0, s)
        if s >= warm:
            tp += attack and flagged
            fp += (not attack) and flagged
            fn += attack and not flagged
    prec = tp / (tp + fp) if tp + fp else 0.0
    rec = tp / (tp + fn) if tp + fn else 0.0
    return 2 * prec * rec / (prec + rec) if prec + rec else 0.0, fp


@pytest.mark.slow
def test_gradient_f1_reference_vs_fixed():
    f1_ref, _ = _f1_run(AttackDetector(compat=True), lambda g: g * 10)
    f1_new, fp_new = _f1_run(AttackDetector(), lambda g: g * 10)
    # BASELINE.md measured 0.702 for the reference at x10 scaling; baseline inflation caps recall
    assert 0.4 < f1_ref < 0.9
    assert f1_new > 0.95 and f1_new > f1_ref
    assert fp_new <= 2


def test_byzantine_median_vs_mean():
    base = torch.randn(1000)
    outs = {0: base + 0.01 * torch.randn(1000), 1: base + 0.01 * torch.randn(1000),
            2: base + 0.01 * torch.randn(1000), 3: -base}
    assert AttackDetector().detect_byzantine_behavior(outs, 0) == [3]
    # reference mean-based rule flags everyone once an outlier exists (A12)
    assert AttackDetector(compat=True).detect_byzantine_behavior(outs, 0) == [0, 1, 2, 3]


def test_backdoor_kl():
    det = AttackDetector()
    a = torch.randn(8, 10)
    assert not det.detect_backdoor_attack(a, a.clone(), 0)
    b = torch.zeros(8, 10)
    b[:, 0] = 50.0
    assert det.detect_backdoor_attack(torch.zeros(8, 10) - b, b, 0)


def test_ml_models_and_exports(tmp_path):
    det = AttackDetector()
    g = torch.Generator().manual_seed(0)
    for s in range(60):
        det.detect_output_anomaly(torch.randn(256, generator=g), 0, s)
    det.update_detection_models()
    assert 0 in det.anomaly_detectors
    stats = det.output_history[0][-1]["stats"]
    assert det.detect_with_ml_models(stats, 0) in (True, False)
    det.export_detection_data(str(tmp_path / "d.json"))
    s = det.get_detection_statistics()
    assert s["nodes_monitored"] == 1 and "f1" in s


def test_ground_truth_counters():
    det = AttackDetector()
    g = torch.Generator().manual_seed(1)
    for s in range(30):
        det.detect_output_anomaly(torch.randn(512, generator=g), 0, s, ground_truth=False)
    det.detect_output_anomaly(torch.randn(512, generator=g) * 5 + 3, 0, 30, ground_truth=True)
    st = det.get_detection_statistics()
    assert st["precision"] == 1.0 and st["recall"] == 1.0


def test_quantiles_propagate_nan_like_numpy():
    """the one-partition quantiles must return NaN for an input holding a NaN, as
    np.median / np.percentile (the reference definitions, attack_detector.py:192-196) do."""
    import numpy as np
    from trustworthy_dl.security.attack_detection import _quantiles, numpy_tensor_statistics
    x = np.random.default_rng(0).standard_normal(1001).astype(np.float32)
    ref = [float(np.percentile(x, 25)), float(np.median(x)), float(np.percentile(x, 75))]
    assert np.allclose(_quantiles(x, (0.25, 0.5, 0.75)), ref)
    x[17] = np.nan
    got = _quantiles(x, (0.25, 0.5, 0.75))
    assert all(np.isnan(v) for v in got) and np.isnan(np.median(x))
    assert np.isnan(numpy_tensor_statistics(x)["median"])
