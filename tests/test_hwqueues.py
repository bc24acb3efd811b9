"""GPU_MAX_HW_QUEUES guard (runtime/hwqueues.py) and the engine's P2P-mode choice (CPU)."""
import os

import pytest

from trustworthy_dl.runtime import hwqueues as hq


@pytest.fixture
def clean(monkeypatch):
    monkeypatch.delenv("TDL_KEEP_HW_QUEUES", raising=False)
    monkeypatch.setattr(hq, "_hip_initialized", lambda: False)
    hq._reset_for_tests()
    yield monkeypatch
    hq._reset_for_tests()


def test_raises_low_queue_count(clean):
    clean.setenv("GPU_MAX_HW_QUEUES", "4")
    assert hq.ensure_hw_queues() == hq.REQUEST_QUEUES
    assert os.environ["GPU_MAX_HW_QUEUES"] == str(hq.REQUEST_QUEUES)
    assert hq.effective_hw_queues() == hq.REQUEST_QUEUES


def test_unset_means_hip_default(clean):
    clean.delenv("GPU_MAX_HW_QUEUES", raising=False)
    assert hq.ensure_hw_queues() == hq.REQUEST_QUEUES


def test_keeps_higher_and_opt_out(clean):
    clean.setenv("GPU_MAX_HW_QUEUES", "32")
    assert hq.ensure_hw_queues(16) == 32
    hq._reset_for_tests()
    clean.setenv("GPU_MAX_HW_QUEUES", "2")
    clean.setenv("TDL_KEEP_HW_QUEUES", "1")
    assert hq.ensure_hw_queues() == 2
    assert os.environ["GPU_MAX_HW_QUEUES"] == "2"


def test_too_late_reports_what_hip_started_with(clean):
    clean.setenv("GPU_MAX_HW_QUEUES", "4")
    clean.setattr(hq, "_hip_initialized", lambda: True)
    assert hq.ensure_hw_queues() == 4
    assert os.environ["GPU_MAX_HW_QUEUES"] == "4"
    assert hq.effective_hw_queues() < hq.ENGINE_QUEUES


def test_engine_p2p_mode_follows_queue_budget(clean):
    """Pre-posted receives only when RCCL streams got queues of their own (parallel/pipeline.py)."""
    import types
    from trustworthy_dl.parallel import pipeline as P
    clean.setattr(P.dist, "get_backend", lambda *a, **k: "nccl")
    fake = types.SimpleNamespace(distributed=True)
    cfg = P.EngineConfig(num_nodes=2)
    clean.setattr(hq, "_effective", 4)
    assert P.PipelineEngine._choose_p2p_mode(fake, cfg) == "grouped"
    clean.setattr(hq, "_effective", 32)
    assert P.PipelineEngine._choose_p2p_mode(fake, cfg) == "async"
    fake.distributed = False                      # local mode: no RCCL, nothing to decide
    clean.setattr(hq, "_effective", 4)
    assert P.PipelineEngine._choose_p2p_mode(fake, cfg) == "async"
