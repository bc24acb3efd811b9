"""Experiment layer on CPU: README-schema YAML configs, synthetic data loaders, NodeMonitor baselines,
ExperimentRunner artefacts (experiment_runner.py:325-591 file set) and the two console entry points."""
import csv
import glob
import json
import os

import numpy as np
import pytest
import torch

from trustworthy_dl.config import load_config
from trustworthy_dl.core.node_monitor import NodeMonitor, gradient_consistency, output_deviation
from trustworthy_dl.utils.data_loader import get_dataloader

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(ROOT, "configs", "*.yaml"))))
def test_every_shipped_config_loads(path):
    cfg, atk, raw = load_config(path)
    assert cfg.num_nodes == raw["distributed"]["num_nodes"]
    assert cfg.model_name == raw["model"]["name"]
    assert isinstance(cfg.learning_rate, float)
    if "security" in raw and "trust_threshold" in raw["security"]:
        assert cfg.trust_threshold == raw["security"]["trust_threshold"]
    assert isinstance(atk.types, list)


def test_readme_schema_fields_and_overrides():
    cfg, _, _ = load_config(os.path.join(ROOT, "configs", "gpt2_distributed.yaml"),
                            {"num_nodes": 2, "batch_size": None})
    assert (cfg.model_name, cfg.model_size, cfg.batch_size) == ("gpt2", "medium", 32)
    assert cfg.learning_rate == pytest.approx(5e-5)          # YAML reads 5e-5 as a string
    assert cfg.num_nodes == 2                                 # override wins, None is ignored
    assert cfg.attack_detection_enabled and cfg.gradient_verification_enabled


def test_dataloaders_shapes_and_determinism():
    lm = list(get_dataloader("openwebtext", "train", 4, seq_len=32, num_batches=2, seed=3))
    assert len(lm) == 2
    b = lm[0]
    assert b["input"].shape == (4, 32) and b["target"].shape == (4, 32) and b["input"].dtype == torch.int64
    again = list(get_dataloader("openwebtext", "train", 4, seq_len=32, num_batches=2, seed=3))
    assert torch.equal(again[0]["input"], b["input"])
    val = next(iter(get_dataloader("openwebtext", "validation", 4, seq_len=32, num_batches=1, seed=3)))
    assert not torch.equal(val["input"], b["input"])           # splits draw different streams
    img = next(iter(get_dataloader("cifar10", "train", 2, num_batches=1)))
    assert img["input"].shape == (2, 3, 32, 32) and int(img["target"].max()) < 10
    big = next(iter(get_dataloader("imagenet", "train", 1, num_batches=1)))
    assert big["input"].shape == (1, 3, 224, 224)
    with pytest.raises(ValueError):
        get_dataloader("no-such-dataset")


def test_node_monitor_baselines_and_scores():
    mon = NodeMonitor(beta=0.5, warmup=2)
    assert mon.get_expected_mean(0) is None and mon.get_expected_gradient_norms(0) == []
    for _ in range(3):
        mon.record_output(0, 1.0, 2.0)
        mon.record_gradient_norms(0, [1.0, 2.0])
    assert mon.get_expected_mean(0) == pytest.approx(1.0)
    assert mon.get_expected_std(0) == pytest.approx(2.0)
    assert np.allclose(mon.get_expected_gradient_norms(0), [1.0, 2.0])
    # reference deviation formula: (|dmean| + |dstd|) / std_exp / 2, clipped to 1
    assert output_deviation(2.0, 2.0, 1.0, 2.0) == pytest.approx(0.25)
    assert output_deviation(100.0, 2.0, 1.0, 2.0) == 1.0
    assert output_deviation(1.0, 1.0, None, None) == 0.0
    # symmetric consistency penalises the x10 poisoned gradient the reference scored 1.0
    assert gradient_consistency([10.0, 20.0], [1.0, 2.0], symmetric=True) < 0.2
    assert gradient_consistency([10.0, 20.0], [1.0, 2.0], symmetric=False) == 1.0
    assert gradient_consistency([], [1.0]) == 0.0 and gradient_consistency([1.0], []) == 1.0
    mon.reset(0)
    assert mon.get_expected_mean(0) is None


@pytest.mark.slow
def test_experiment_runner_writes_reference_artifacts(tmp_path):
    from trustworthy_dl.experiments.runner import ExperimentConfig, ExperimentRunner
    cfg = ExperimentConfig(experiment_name="tiny", model_name="gpt2", dataset_name="openwebtext", num_nodes=2,
                           num_epochs=2, batch_size=4, learning_rate=1e-3, attack_enabled=True,
                           attack_start_epoch=1, attack_target_nodes=[1], batches_per_epoch=3,
                           model_size="tiny", seq_len=32, micro_batches=2, device="cpu",
                           output_dir=str(tmp_path), save_interval=1)
    res = ExperimentRunner(cfg).run_experiment()
    out = tmp_path / "tiny"
    for name in ("experiment_results.json", "training_metrics.csv", "experiment_report.md"):
        assert (out / name).exists(), name
    data = json.loads((out / "experiment_results.json").read_text())
    for key in ("experiment_config", "training_results", "final_trust_statistics", "experiment_summary"):
        assert key in data and key in res, key
    rows = list(csv.DictReader(open(out / "training_metrics.csv")))
    assert rows and set(rows[0]) == {"epoch", "batch", "loss", "timestamp"}
    assert all(np.isfinite(float(r["loss"])) for r in rows)
    summary = data["experiment_summary"]
    assert summary["total_batches"] == 6
    assert "final_system_trust" in summary


def test_train_cli_runs_a_config(tmp_path):
    from trustworthy_dl import cli
    stats = cli.main(["--config", os.path.join(ROOT, "configs", "gpt2_distributed.yaml"), "--size", "tiny",
                   "--nodes", "2", "--epochs", "1", "--batch-size", "4", "--seq-len", "32",
                   "--micro-batches", "2", "--batches-per-epoch", "2", "--device", "cpu",
                   "--checkpoint-dir", str(tmp_path / "ckpt")])
    # get_training_stats() schema (distributed_trainer.py:510-521), after 1 epoch x 2 batches
    for key in ("current_epoch", "global_step", "training_state", "trust_scores", "attack_count", "metrics"):
        assert key in stats, key
    assert stats["global_step"] == 2
