"""Experiment orchestration: ``ExperimentConfig``, ``ExperimentRunner``, ``main``.

Parity target: reference experiment_runner.py:31-633 — same config fields and defaults, same
artifact names (``experiment_results.json``, ``training_metrics.csv``,
``intermediate_epoch_{e}.json``, ``training_loss.png``, ``trust_evolution.png``,
``attack_impact.png``, ``system_metrics.png``, ``experiment_report.md``) and CLI flags
(``--config --model --dataset --nodes --epochs --attack``).  Unlike the reference, which
simulates the loss, trust curves, memory and utilisation with ``np.random``
(experiment_runner.py:201-216, 262-268, 385-451), every number here is measured:
the runner drives the real ``DistributedTrainer`` step by step, the attacker injects real faults
and the detection / trust / system curves are recorded from the engine.  ``--config`` is honoured
(A19).  Plots need matplotlib; without it the PNGs are skipped and the rest is still written.
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import time
from dataclasses import asdict, dataclass, field
from datetime import datetime
from pathlib import Path
from typing import Any, Dict, List, Optional

import numpy as np

from ..attacks import AdversarialAttacker, AttackConfig
from ..config import TrainingConfig, load_config
from ..core.distributed_trainer import DistributedTrainer
from ..utils.data_loader import get_dataloader
from ..utils.metrics import MetricsCollector

logger = logging.getLogger(__name__)


@dataclass
class ExperimentConfig:
    experiment_name: str
    model_name: str
    dataset_name: str
    num_nodes: int
    num_epochs: int
    batch_size: int
    learning_rate: float
    attack_enabled: bool = True
    attack_start_epoch: int = 2
    attack_intensity: float = 0.5
    trust_threshold: float = 0.7
    save_interval: int = 100
    output_dir: str = "results"
    # ---- extensions
    attack_types: List[str] = field(default_factory=lambda: ["gradient_poisoning", "data_poisoning"])
    attack_target_nodes: List[int] = field(default_factory=lambda: [1, 3])
    attack_probability: float = 1.0
    steps_per_epoch_estimate: int = 100
    batches_per_epoch: int = 20
    model_size: Optional[str] = None
    seq_len: int = 128
    micro_batches: int = 2
    device: str = "auto"
    reassignment_enabled: bool = True
    seed: int = 0


class ExperimentRunner:
    def __init__(self, config: ExperimentConfig, training_config: Optional[TrainingConfig] = None):
        self.config = config
        self.output_dir = Path(config.output_dir) / config.experiment_name
        self.output_dir.mkdir(parents=True, exist_ok=True)
        self.metrics_collector = MetricsCollector()
        self.results_data = {"training_metrics": [], "trust_metrics": [], "attack_metrics": [], "system_metrics": []}
        self.training_config = training_config or TrainingConfig(
            model_name=config.model_name, dataset_name=config.dataset_name, batch_size=config.batch_size,
            learning_rate=config.learning_rate, num_epochs=config.num_epochs, num_nodes=config.num_nodes,
            trust_threshold=config.trust_threshold, model_size=config.model_size, seq_len=config.seq_len,
            micro_batches=config.micro_batches, device=config.device, checkpoint_interval=0,
            reassignment_enabled=config.reassignment_enabled, batches_per_epoch=config.batches_per_epoch,
            seed=config.seed, checkpoint_dir=str(self.output_dir / "checkpoints"))
        self.trainer: Optional[DistributedTrainer] = None
        self.attacker: Optional[AdversarialAttacker] = None
        logger.info("ExperimentRunner initialized: %s", config.experiment_name)

    # ------------------------------------------------------------------ setup
    def setup_experiment(self):
        c = self.config
        if c.attack_enabled:
            # start_step = attack_start_epoch * steps/epoch (experiment_runner.py:95 used a fixed 100)
            start = c.attack_start_epoch * c.batches_per_epoch
            self.attacker = AdversarialAttacker(AttackConfig(
                attack_types=list(c.attack_types), target_nodes=list(c.attack_target_nodes),
                intensity=c.attack_intensity, start_step=start, probability=c.attack_probability, seed=c.seed))
        self.trainer = DistributedTrainer(self.training_config, attacker=self.attacker)
        self.trainer.create_model_partitions()
        kw = {"seq_len": self.training_config.seq_len, "seed": c.seed}
        self.train_loader = get_dataloader(c.dataset_name, "train", c.batch_size,
                                           num_batches=c.batches_per_epoch, **kw)
        self.val_loader = get_dataloader(c.dataset_name, "validation", c.batch_size, num_batches=2, **kw)
        logger.info("Experiment setup completed")

    # ------------------------------------------------------------------ run
    def run_experiment(self) -> Dict[str, Any]:
        logger.info("Starting experiment: %s", self.config.experiment_name)
        t0 = time.time()
        try:
            self.setup_experiment()
            training_results = self._run_training_with_monitoring()
            final = self._collect_final_results(training_results)
            self._save_results(final)
            self._generate_visualizations()
            self._generate_experiment_report(final)
            logger.info("Experiment completed in %.2f seconds", time.time() - t0)
            return final
        except Exception as e:  # pragma: no cover - surfaced to the caller
            logger.error("Experiment failed: %s", e)
            raise
        finally:
            self._cleanup()

    def _run_training_with_monitoring(self) -> Dict[str, Any]:
        c = self.config
        training_metrics = []
        for epoch in range(c.num_epochs):
            t0 = time.time()
            if c.attack_enabled and epoch >= c.attack_start_epoch and self.attacker and not self.attacker.is_active():
                self.attacker.activate_attacks()
            loss = self._run_epoch(epoch)
            em = self._collect_epoch_metrics(epoch, loss, time.time() - t0)
            training_metrics.append(em)
            logger.info("Epoch %d/%d - Loss: %.4f - Time: %.2fs", epoch + 1, c.num_epochs, loss, time.time() - t0)
            if (epoch + 1) % 5 == 0:
                self._save_intermediate_results(training_metrics, epoch)
        return {"training_metrics": training_metrics}

    def _run_epoch(self, epoch: int) -> float:
        tr = self.trainer
        eng = tr.engine
        eng.epoch = epoch
        tr.current_epoch = epoch
        n0 = len(tr.metrics_collector.batch_metrics)
        for batch_idx, batch in enumerate(self.train_loader):
            eng.train_step(batch)
        eng.flush()
        new = tr.metrics_collector.batch_metrics[n0:]
        for i, m in enumerate(new):
            if m.get("loss") is None:
                continue
            if i % max(1, self.config.save_interval) == 0:   # experiment_runner.py:196
                self._collect_batch_metrics(epoch, m.get("step", i), m["loss"], m)
        losses = [m["loss"] for m in new if m.get("loss") is not None]
        return float(np.mean(losses)) if losses else float("nan")

    def _collect_batch_metrics(self, epoch: int, batch_idx: int, loss: float, extra: Optional[Dict] = None):
        rec = {"epoch": epoch, "batch": batch_idx, "loss": loss, "timestamp": time.time()}
        self.results_data["training_metrics"].append(rec)
        if extra and "trust_scores" in extra:
            self.results_data["trust_metrics"].append({"step": batch_idx, "epoch": epoch,
                                                       **{f"node_{k}": v for k, v in extra["trust_scores"].items()}})

    def _collect_epoch_metrics(self, epoch: int, epoch_loss: float, epoch_time: float) -> Dict[str, Any]:
        tm = self.trainer.trust_manager
        n = self.config.num_nodes
        attack = self.attacker.get_attack_statistics() if self.attacker else {}
        system = {"memory": MetricsCollector.device_memory(), "epoch_time_s": epoch_time,
                  "communication_overhead": self._estimate_communication_overhead(),
                  "gpu_utilization": self._get_gpu_utilization(),
                  "pipeline_busy_fraction": self._pipeline_busy_fraction(),
                  "gpu": MetricsCollector.gpu_system_metrics()}
        self.results_data["attack_metrics"].append({"epoch": epoch, **{k: v for k, v in attack.items()
                                                                        if not isinstance(v, (list, dict))}})
        self.results_data["system_metrics"].append({"epoch": epoch, **system})
        return {"epoch": epoch, "timestamp": time.time(), "training_loss": epoch_loss,
                "trust_scores": {i: tm.get_trust_score(i) for i in range(n)},
                "node_statuses": {i: tm.get_node_status(i).value for i in range(n)},
                "attack_metrics": attack, "system_metrics": system,
                "plan": self.trainer.engine.plan.describe()}

    def _get_memory_usage(self) -> float:
        mem = MetricsCollector.device_memory()
        return float(mem.get("hbm_used_fraction", 0.0))

    def _get_gpu_utilization(self) -> float:
        """Device busy fraction from the amdgpu driver (sysfs ``gpu_busy_percent``, the counter
        rocm-smi reports); on hosts without one, the pipeline busy fraction below."""
        m = MetricsCollector.gpu_system_metrics()
        if "gpu_busy_percent" in m:
            return m["gpu_busy_percent"] / 100.0
        return self._pipeline_busy_fraction()

    def _pipeline_busy_fraction(self) -> float:
        """Fraction of step time not spent blocked in pipeline communication (host-measured)."""
        e = self.trainer.engine
        return 1.0 - (e._comm_wait / e._step_time) if e._step_time > 0 else 0.0

    def _estimate_communication_overhead(self) -> float:
        e = self.trainer.engine
        return e._comm_wait / e._step_time if e._step_time > 0 else 0.0

    # ------------------------------------------------------------------ results
    def _collect_final_results(self, training_results: Dict) -> Dict[str, Any]:
        return {
            "experiment_config": asdict(self.config),
            "training_config": asdict(self.training_config),
            "training_results": training_results,
            "final_trust_statistics": self.trainer.trust_manager.get_trust_statistics(),
            "final_attack_statistics": self.attacker.get_final_statistics() if self.attacker else {},
            "detection_statistics": self.trainer.attack_detector.get_detection_statistics(),
            "attack_history": self.trainer.attack_history,
            "reassignment_history": self.trainer.reassignment_history,
            "results_data": self.results_data,
            "experiment_summary": self._generate_experiment_summary(),
        }

    def _generate_experiment_summary(self) -> Dict[str, Any]:
        tm = self.results_data["training_metrics"]
        if not tm:
            return {}
        losses = [m["loss"] for m in tm]
        s = {"total_batches": len(tm), "average_loss": float(np.mean(losses)), "final_loss": losses[-1],
             "loss_reduction": (losses[0] - losses[-1]) / losses[0] if len(losses) > 1 else 0.0,
             "convergence_achieved": losses[-1] < 0.5}
        ts = self.trainer.trust_manager.get_trust_statistics()
        s.update({"final_system_trust": ts.get("system_trust", 0.0),
                  "compromised_nodes": len(self.trainer.trust_manager.get_compromised_nodes()),
                  "total_attacks_detected": len(self.trainer.attack_history),
                  "reassignments": len(self.trainer.reassignment_history)})
        if self.attacker:
            s.update({k: v for k, v in self.attacker.detection_metrics().items() if not isinstance(v, dict)})
        return s

    def _save_results(self, results: Dict[str, Any]):
        with open(self.output_dir / "experiment_results.json", "w") as f:
            json.dump(results, f, indent=2, default=str)
        rows = self.results_data["training_metrics"]
        if rows:
            import csv
            with open(self.output_dir / "training_metrics.csv", "w", newline="") as f:
                w = csv.DictWriter(f, fieldnames=["epoch", "batch", "loss", "timestamp"])
                w.writeheader()
                for r in rows:
                    w.writerow({k: r[k] for k in ("epoch", "batch", "loss", "timestamp")})
        self.trainer.trust_manager.export_trust_data(str(self.output_dir / "trust_data.json"))
        self.trainer.attack_detector.export_detection_data(str(self.output_dir / "detection_data.json"))

    def _save_intermediate_results(self, metrics: List[Dict], epoch: int):
        with open(self.output_dir / f"intermediate_epoch_{epoch}.json", "w") as f:
            json.dump(metrics, f, indent=2, default=str)

    # ------------------------------------------------------------------ plots (measured data)
    def _generate_visualizations(self):
        try:
            import matplotlib
            matplotlib.use("Agg")
            import matplotlib.pyplot as plt  # noqa: F401
        except Exception:
            logger.warning("matplotlib not available: skipping PNG plots")
            return
        self._plot_training_loss()
        self._plot_trust_evolution()
        self._plot_attack_impact()
        self._plot_system_metrics()

    def _plot_training_loss(self):
        import matplotlib.pyplot as plt
        tm = self.results_data["training_metrics"]
        if not tm:
            return
        steps = [m["batch"] for m in tm]
        plt.figure(figsize=(10, 5))
        plt.plot(steps, [m["loss"] for m in tm], "b-", alpha=0.7, label="training loss")
        for r in self.trainer.reassignment_history:
            plt.axvline(r["step"], color="r", ls="--", alpha=0.6)
        plt.xlabel("step")
        plt.ylabel("loss")
        plt.legend()
        plt.grid(alpha=0.3)
        plt.savefig(self.output_dir / "training_loss.png", dpi=120, bbox_inches="tight")
        plt.close()

    def _plot_trust_evolution(self):
        import matplotlib.pyplot as plt
        tr = self.results_data["trust_metrics"]
        if not tr:
            return
        plt.figure(figsize=(10, 6))
        steps = [r["step"] for r in tr]
        for n in range(self.config.num_nodes):
            plt.plot(steps, [r.get(f"node_{n}", np.nan) for r in tr], label=f"node {n}", lw=2)
        plt.axhline(self.config.trust_threshold, color="k", ls=":", label="threshold")
        plt.ylim(0, 1.05)
        plt.xlabel("step")
        plt.ylabel("trust score")
        plt.legend()
        plt.grid(alpha=0.3)
        plt.savefig(self.output_dir / "trust_evolution.png", dpi=120, bbox_inches="tight")
        plt.close()

    def _plot_attack_impact(self):
        import matplotlib.pyplot as plt
        am = self.results_data["attack_metrics"]
        if not am:
            return
        ep = [a["epoch"] for a in am]
        fig, ax = plt.subplots(1, 3, figsize=(15, 4))
        ax[0].plot(ep, [a.get("recall", 0) for a in am], "g-o")
        ax[0].set_title("detection recall (cumulative)")
        ax[1].plot(ep, [a.get("precision", 0) for a in am], "b-o")
        ax[1].set_title("detection precision (cumulative)")
        ax[2].plot(ep, [a.get("total_injections", 0) for a in am], "r-o")
        ax[2].set_title("injected attacks (cumulative)")
        for a in ax:
            a.set_xlabel("epoch")
            a.grid(alpha=0.3)
        plt.tight_layout()
        plt.savefig(self.output_dir / "attack_impact.png", dpi=120, bbox_inches="tight")
        plt.close()

    def _plot_system_metrics(self):
        import matplotlib.pyplot as plt
        sm = self.results_data["system_metrics"]
        if not sm:
            return
        ep = [s["epoch"] for s in sm]
        fig, ax = plt.subplots(1, 3, figsize=(15, 4))
        ax[0].plot(ep, [s["memory"].get("max_allocated_gb", 0) for s in sm], "b-o")
        ax[0].set_title("peak device memory (GB)")
        ax[1].plot(ep, [s["gpu_utilization"] for s in sm], "g-o")
        ax[1].set_title("utilization (1 - comm wait / step)")
        ax[2].plot(ep, [s["communication_overhead"] for s in sm], "r-o")
        ax[2].set_title("communication overhead")
        for a in ax:
            a.set_xlabel("epoch")
            a.grid(alpha=0.3)
        plt.tight_layout()
        plt.savefig(self.output_dir / "system_metrics.png", dpi=120, bbox_inches="tight")
        plt.close()

    # ------------------------------------------------------------------ report
    def _generate_experiment_report(self, results: Dict[str, Any]):
        with open(self.output_dir / "experiment_report.md", "w") as f:
            f.write(self._create_report_content(results))

    def _create_report_content(self, results: Dict[str, Any]) -> str:
        s = results.get("experiment_summary", {})
        c = self.config
        fmt = lambda v, spec: format(v, spec) if isinstance(v, (int, float)) else str(v)  # noqa: E731
        lines = [f"# Experiment Report: {c.experiment_name}", "", "## Configuration",
                 f"- Model: {c.model_name}", f"- Dataset: {c.dataset_name} (synthetic)", f"- Nodes: {c.num_nodes}",
                 f"- Epochs: {c.num_epochs}", f"- Batch size: {c.batch_size}", f"- Learning rate: {c.learning_rate}",
                 f"- Attacks enabled: {c.attack_enabled} ({', '.join(c.attack_types)} on nodes {c.attack_target_nodes}, "
                 f"intensity {c.attack_intensity}, from epoch {c.attack_start_epoch})",
                 f"- Trust threshold: {c.trust_threshold}", "", "## Results (measured)", "",
                 "### Training", f"- Total batches: {s.get('total_batches', 'N/A')}",
                 f"- Average loss: {fmt(s.get('average_loss', 'N/A'), '.4f')}",
                 f"- Final loss: {fmt(s.get('final_loss', 'N/A'), '.4f')}",
                 f"- Loss reduction: {fmt(s.get('loss_reduction', 'N/A'), '.2%')}", "",
                 "### Security", f"- Final system trust: {fmt(s.get('final_system_trust', 'N/A'), '.3f')}",
                 f"- Compromised nodes: {s.get('compromised_nodes', 'N/A')}",
                 f"- Attacks detected: {s.get('total_attacks_detected', 'N/A')}",
                 f"- Task reassignments: {s.get('reassignments', 'N/A')}"]
        if "f1" in s:
            lines += [f"- Detection precision / recall / F1: {s['precision']:.3f} / {s['recall']:.3f} / {s['f1']:.3f}",
                      f"- Mean time to detect: {s.get('mean_time_to_detect_steps')} steps"]
        lines += ["", "### Reassignments"]
        for r in self.trainer.reassignment_history:
            lines.append(f"- step {r['step']}: nodes {r['from_nodes']} excluded -> {r['plan']} "
                         f"(migration {r['migration_time'] * 1000:.1f} ms, {r['moved_params']} params)")
        lines += ["", "## Artifacts", "- `experiment_results.json`, `training_metrics.csv`, `trust_data.json`, "
                  "`detection_data.json`", "- `training_loss.png`, `trust_evolution.png`, `attack_impact.png`, "
                  "`system_metrics.png`", "", f"*Report generated on {datetime.now():%Y-%m-%d %H:%M:%S}*", ""]
        return "\n".join(lines)

    def _cleanup(self):
        if self.trainer:
            self.trainer.cleanup()
        if self.attacker:
            self.attacker.cleanup()


def build_arg_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Run trustworthy distributed DL experiments")
    p.add_argument("--config", type=str, help="README-schema YAML config (honoured)")
    p.add_argument("--model", type=str, default="gpt2")
    p.add_argument("--dataset", type=str, default="openwebtext")
    p.add_argument("--nodes", type=int, default=4)
    p.add_argument("--epochs", type=int, default=10)
    p.add_argument("--attack", action="store_true")
    p.add_argument("--batch-size", type=int, default=32)
    p.add_argument("--lr", type=float, default=5e-5)
    p.add_argument("--batches-per-epoch", type=int, default=20)
    p.add_argument("--seq-len", type=int, default=128)
    p.add_argument("--output-dir", type=str, default="results")
    p.add_argument("--device", type=str, default="auto")
    return p


def main(argv=None):
    logging.basicConfig(level=logging.INFO)
    args = build_arg_parser().parse_args(argv)
    tc = None
    attack_types, targets, intensity, start = ["gradient_poisoning", "data_poisoning"], [1, 3], 0.5, 2
    if args.config:
        tc, atk, _ = load_config(args.config)
        args.model, args.dataset, args.nodes, args.epochs = tc.model_name, tc.dataset_name, tc.num_nodes, tc.num_epochs
        args.batch_size, args.lr = tc.batch_size, tc.learning_rate
        args.attack = args.attack or atk.enabled
        attack_types, targets, intensity = atk.types, atk.target_nodes, atk.intensity
    name = f"{args.model}_{args.dataset}_nodes{args.nodes}_{datetime.now():%Y%m%d_%H%M%S}"
    cfg = ExperimentConfig(experiment_name=name, model_name=args.model, dataset_name=args.dataset, num_nodes=args.nodes,
                           num_epochs=args.epochs, batch_size=args.batch_size, learning_rate=args.lr,
                           attack_enabled=args.attack, attack_types=attack_types,
                           attack_target_nodes=[t for t in targets if t < args.nodes] or [args.nodes - 1],
                           attack_intensity=intensity, attack_start_epoch=min(start, max(0, args.epochs - 1)),
                           batches_per_epoch=args.batches_per_epoch, seq_len=args.seq_len, output_dir=args.output_dir,
                           device=args.device)
    runner = ExperimentRunner(cfg, tc)
    if tc is not None:
        runner.training_config.batches_per_epoch = args.batches_per_epoch
        runner.training_config.checkpoint_dir = str(runner.output_dir / "checkpoints")
        runner.training_config.checkpoint_interval = 0
    runner.run_experiment()
    print(f"Experiment completed: {cfg.experiment_name}")
    print(f"Results saved to: {runner.output_dir}")
    return runner


if __name__ == "__main__":
    main()
