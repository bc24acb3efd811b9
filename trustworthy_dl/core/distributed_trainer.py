"""``DistributedTrainer`` — the reference's training orchestrator API on the trust-aware pipeline engine.

Reference: distributed_trainer.py:30-527 (TrainingState, NodeConfig, TrainingConfig,
DistributedTrainer).  Every public method is kept; the ones the reference leaves broken or
simulated are real here: partitions include embeddings / head / remainder
layers (A2), compromised stages are re-sharded instead of silently skipped (A4, A6), optimizers
exist and step (A5), checkpoints create their directory and can be loaded (A7), the LM loss is on
real logits (A8), validation has no detector side effects (A21) and the process group is actually
set up (A22).  The README facade ``DistributedTrainer(model_name=..., num_nodes=...,
trust_threshold=...)`` / ``train(dataset=..., epochs=..., trust_manager=...)`` is supported (A20).
"""
from __future__ import annotations

import logging
import os
import time
from dataclasses import asdict, dataclass
from enum import Enum
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..config import TrainingConfig
from ..models import get_model
from ..parallel.flat import AdamWConfig
from ..parallel.pipeline import EngineConfig, PipelineEngine
from ..runtime import faults
from ..security.attack_detection import AttackDetector
from ..security.gradient_verification import GradientVerifier
from ..utils.metrics import MetricsCollector
from .node_monitor import NodeMonitor, gradient_consistency, output_deviation
from .trust_manager import NodeStatus, TrustManager

logger = logging.getLogger(__name__)

__all__ = ["TrainingState", "NodeConfig", "TrainingConfig", "DistributedTrainer"]


class TrainingState(Enum):
    INITIALIZING = "initializing"
    TRAINING = "training"
    UNDER_ATTACK = "under_attack"
    RECOVERING = "recovering"
    COMPLETED = "completed"


@dataclass
class NodeConfig:
    """Per-node placement record (distributed_trainer.py:37-46), populated from the live plan."""
    node_id: int
    rank: int
    world_size: int
    gpu_id: int
    model_partition: str
    trust_score: float = 1.0
    status: NodeStatus = NodeStatus.TRUSTED


class DistributedTrainer:
    def __init__(self, config: Optional[TrainingConfig] = None, *, model_name: Optional[str] = None,
                 num_nodes: Optional[int] = None, trust_threshold: Optional[float] = None,
                 trust_manager: Optional[TrustManager] = None, attacker=None, **kwargs):
        if config is None:
            config = TrainingConfig()
        overrides = {"model_name": model_name, "num_nodes": num_nodes, "trust_threshold": trust_threshold, **kwargs}
        for k, v in overrides.items():
            if v is not None and hasattr(config, k):
                setattr(config, k, v)
        self.config = config
        self.training_state = TrainingState.INITIALIZING
        self.current_epoch = 0
        self.epoch_batch = 0          # batches of current_epoch already trained (resume position)
        self.trust_manager = trust_manager or TrustManager(num_nodes=config.num_nodes,
                                                           trust_threshold=config.trust_threshold)
        self.node_monitor = NodeMonitor()
        self.attack_detector = AttackDetector()
        self.gradient_verifier = GradientVerifier(self.attack_detector)
        self.metrics_collector = MetricsCollector()
        self.attacker = attacker
        self.node_configs: Dict[int, NodeConfig] = {}
        self.model_partitions: Dict[int, torch.nn.Module] = {}
        self.optimizers: Dict[int, Any] = {}
        self.schedulers: Dict[int, Any] = {}
        self.engine: Optional[PipelineEngine] = None
        self._owns_pg = False
        self._phase_open = False      # per-phase API: a step opened by forward_pass, closed by optimizer_step
        self._phase_loss: Optional[torch.Tensor] = None
        logger.info("Initialized DistributedTrainer with %d nodes", config.num_nodes)

    # ------------------------------------------------------------------ properties mirroring engine state
    @property
    def global_step(self) -> int:
        return self.engine.global_step if self.engine else 0

    @property
    def attack_history(self) -> List[Dict]:
        return self.engine.attack_history if self.engine else []

    @property
    def reassignment_history(self) -> List[Dict]:
        return self.engine.reassignment_history if self.engine else []

    # ------------------------------------------------------------------ distributed bring-up
    def setup_distributed_environment(self, rank: int, world_size: int, backend: Optional[str] = None,
                                      master_addr: Optional[str] = None, master_port: Optional[int] = None):
        """Process group over RCCL (GPU) or gloo (CPU) + device binding (distributed_trainer.py:99-114)."""
        os.environ.setdefault("MASTER_ADDR", master_addr or "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(master_port or 12355))
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if not dist.is_initialized():
            kw = {}
            if backend == "nccl":
                local = int(os.environ.get("LOCAL_RANK", rank % max(1, torch.cuda.device_count())))
                torch.cuda.set_device(local)
                kw["device_id"] = torch.device("cuda", local)
            dist.init_process_group(backend=backend, rank=rank, world_size=world_size, **kw)
            self._owns_pg = True
        self.config.num_nodes = world_size
        self.trust_manager.resize(world_size)
        logger.info("Initialized distributed environment: rank %d/%d (%s)", rank, world_size, backend)

    # ------------------------------------------------------------------ model / partitions
    def _engine_config(self) -> EngineConfig:
        c = self.config
        return EngineConfig(
            num_nodes=c.num_nodes, micro_batches=c.micro_batches, compute_dtype=c.compute_dtype, device=c.device,
            seq_len=c.seq_len,
            adamw=AdamWConfig(lr=c.learning_rate, betas=tuple(c.adam_betas), weight_decay=c.weight_decay,
                              max_grad_norm=c.max_grad_norm),
            attack_detection=c.attack_detection_enabled, gradient_verification=c.gradient_verification_enabled,
            quarantine=c.quarantine_enabled, verifier=dict(c.verifier), trust_threshold=c.trust_threshold,
            trust_decay_per_step=c.trust_decay_per_step, reassign=c.reassignment_enabled,
            max_reassignment_attempts=c.max_reassignment_attempts, seed=c.seed,
            data_parallel=c.data_parallel, defer_wgrad=c.defer_wgrad,
            layer_granularity=c.layer_granularity, heartbeat_interval=c.heartbeat_interval,
            heartbeat_timeout=c.heartbeat_timeout, abort_on_offline=c.abort_on_offline)

    def create_model_partitions(self, model_name: Optional[str] = None) -> Dict[int, torch.nn.Module]:
        """Build the model, plan a cost-balanced partition over the nodes and instantiate the stages
        this process owns (distributed_trainer.py:116-146)."""
        c = self.config
        name = model_name or c.model_name
        kw = {}
        if name.startswith("gpt"):
            kw["seq_len"] = c.seq_len
            if c.model_size:
                kw["size"] = c.model_size
        if c.num_classes:
            kw["num_classes"] = c.num_classes
        if c.image_size:
            kw["image_size"] = c.image_size
        model = get_model(name, seed=c.seed, **kw)
        self.engine = PipelineEngine(model, self._engine_config(), trust_manager=self.trust_manager,
                                     attacker=self.attacker, metrics=self.metrics_collector,
                                     detector=self.attack_detector)
        self._sync_partitions()
        return self.model_partitions

    def _sync_partitions(self):
        e = self.engine
        self.model_partitions = {n: st.module for n, st in e.stages.items()}
        self.optimizers = {n: st.flat for n, st in e.stages.items()}
        world = e.world
        self.node_configs = {}
        for sid, (node, (a, b)) in enumerate(zip(e.plan.ranks, e.plan.ranges)):
            dev = e._stage_device(node)
            self.node_configs[node] = NodeConfig(node, node, world, dev.index if dev.index is not None else -1,
                                                 f"layers[{a}:{b}]", self.trust_manager.get_trust_score(node),
                                                 self.trust_manager.get_node_status(node))

    def _ensure_engine(self):
        if self.engine is None:
            self.create_model_partitions()

    # ------------------------------------------------------------------ per-phase reference API (local mode)
    def forward_pass(self, inputs: torch.Tensor, node_sequence: Optional[Sequence[int]] = None,
                     labels: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, Dict[int, torch.Tensor]]:
        """Sequential pass over this process's stages, returning (output, per-node outputs)
        (distributed_trainer.py:148-175).  Compromised nodes are NOT skipped (A4): their layers
        are re-sharded by ``reassign_node_tasks`` instead."""
        self._ensure_engine()
        e = self.engine
        if not self._phase_open:       # first phase of a reference-style step
            e.begin_step()
            self._phase_open = True
            self._phase_loss = None
        seq = list(node_sequence) if node_sequence is not None else list(e.plan.ranks)
        x = inputs
        outs = {}
        for k, node in enumerate(seq):
            st = e.stages.get(node)
            if st is None:
                continue
            x = e._stage_input(x, st) if k == 0 else x.to(st.device)
            seen = []
            y, mon = st.forward(x, labels.to(st.device) if (st.computes_loss and labels is not None) else None,
                                observe=lambda t: seen.append(t.detach().clone()))
            if mon is None and seen:
                mon = seen[0]  # the fused LM head reuses its logits buffer: keep a copy
            outs[node] = mon if mon is not None else y
            if self.config.attack_detection_enabled and outs[node] is not None:
                if self.attack_detector.detect_output_anomaly(outs[node], node, e.global_step):
                    self.handle_detected_attack(node, outs[node])
            x = y
        return x, outs

    def backward_pass(self, loss: torch.Tensor, node_sequence: Optional[Sequence[int]] = None) -> Dict[int, List[torch.Tensor]]:
        """loss.backward() then per-node gradient verification (distributed_trainer.py:177-207)."""
        self._ensure_engine()
        loss.backward()
        self._phase_loss = loss.detach() if self._phase_loss is None else self._phase_loss + loss.detach()
        grads = {}
        for node in reversed(list(node_sequence) if node_sequence is not None else list(self.engine.plan.ranks)):
            st = self.engine.stages.get(node)
            if st is None:
                continue
            g = [st.flat.view(st.flat.grad, i) for i in range(len(st.flat.params))]
            grads[node] = g
            if self.config.gradient_verification_enabled:
                if not self.gradient_verifier.verify_gradients(g, node, self.engine.global_step):
                    self.handle_gradient_attack(node, g)
        return grads

    def update_trust_scores(self, node_outputs: Dict[int, torch.Tensor], gradients: Dict[int, List[torch.Tensor]]):
        """Host trust update from monitored outputs / gradients (distributed_trainer.py:209-226)."""
        for node in range(self.config.num_nodes):
            od = self.calculate_output_deviation(node_outputs.get(node), node)
            gc = self.calculate_gradient_consistency(gradients.get(node), node)
            self.trust_manager.update_trust_score(node, od, gc, **self.node_monitor.runtime_metrics(node))

    def calculate_output_deviation(self, output: Optional[torch.Tensor], node_id: int) -> float:
        if output is None:
            return 1.0
        o = output.detach().float()
        mean, std = float(o.mean()), float(o.std())
        dev = output_deviation(mean, std, self.node_monitor.get_expected_mean(node_id),
                               self.node_monitor.get_expected_std(node_id))
        self.node_monitor.record_output(node_id, mean, std)
        return dev

    def calculate_gradient_consistency(self, gradients: Optional[List[torch.Tensor]], node_id: int) -> float:
        if not gradients:
            return 0.0
        norms = [float(g.float().norm()) for g in gradients]
        score = gradient_consistency(norms, self.node_monitor.get_expected_gradient_norms(node_id), symmetric=True)
        self.node_monitor.record_gradient_norms(node_id, norms)
        return score

    def handle_detected_attack(self, node_id: int, output: torch.Tensor):
        """Record + compromise + reassign (distributed_trainer.py:273-299)."""
        o = output.detach().float()
        rec = {"node_id": node_id, "timestamp": time.time(), "step": self.global_step, "attack_type": "output_anomaly",
               "output_stats": {"mean": float(o.mean()), "std": float(o.std()), "max": float(o.max()),
                                "min": float(o.min())}}
        self.attack_history.append(rec)
        self.trust_manager.mark_compromised(node_id, "output_anomaly")
        self.reassign_node_tasks(node_id)
        self.training_state = TrainingState.UNDER_ATTACK

    def handle_gradient_attack(self, node_id: int, gradients: List[torch.Tensor]):
        """distributed_trainer.py:301-322 (also sets UNDER_ATTACK, unlike the reference)."""
        rec = {"node_id": node_id, "timestamp": time.time(), "step": self.global_step,
               "attack_type": "gradient_poisoning",
               "gradient_stats": {"norms": [float(g.float().norm()) for g in gradients],
                                  "num_gradients": len(gradients)}}
        self.attack_history.append(rec)
        self.trust_manager.mark_compromised(node_id, "gradient_poisoning")
        self.reassign_node_tasks(node_id)
        self.training_state = TrainingState.UNDER_ATTACK

    def reassign_node_tasks(self, compromised_node_id: int):
        """Re-shard the compromised node's layers over the trusted nodes (distributed_trainer.py:324-352)."""
        self._ensure_engine()
        if not self.config.reassignment_enabled:
            return
        trusted = [n for n in self.engine.plan.ranks if n != compromised_node_id]
        if not trusted:
            logger.error("No trusted nodes available for reassignment")
            return
        self.engine.reassign([compromised_node_id])
        self._sync_partitions()

    def estimate_migration_time(self, source_node: int, target_node: Optional[int] = None) -> float:
        self._ensure_engine()
        a, b = self.engine.plan.layers_of_rank(source_node)
        numel = sum(self.engine._layer_numel(li) for li in range(a, b))
        return self.engine.estimate_migration_time(numel)

    def perform_task_reassignment(self, source_node: int, target_node: Optional[int] = None):
        self.reassign_node_tasks(source_node)

    # ------------------------------------------------------------------ training
    def calculate_loss(self, outputs: torch.Tensor, targets: torch.Tensor) -> torch.Tensor:
        from ..ops import cross_entropy
        if outputs.dim() == 0:
            return outputs  # loss stages already return the loss
        # GPT-2 logits carry the padded vocabulary rows (50257 -> 50304): the softmax covers the
        # real classes only, as the fused LM-head loss of train_step does
        cfg = getattr(self.engine.model, "config", None) if self.engine is not None else None
        ncls = getattr(cfg, "vocab_size", None) or self.config.num_classes
        return cross_entropy(outputs.reshape(-1, outputs.shape[-1]), targets.reshape(-1), ncls)

    def optimizer_step(self, gradients=None) -> Optional[float]:
        """Apply the step whose gradients ``backward_pass`` accumulated (distributed_trainer.py:441-446):
        tied-weight reduction, device verification digest + quarantine, global-norm clipping and
        the fused AdamW on every local stage — the tail ``train_step`` runs, so the per-phase loop
        and ``train_step`` update the weights identically.  ``gradients`` is accepted for API
        parity; the engine reads the stages' flat gradient buffers directly.  Returns the loss."""
        self._ensure_engine()
        if not self._phase_open:
            return None
        loss = self._phase_loss
        self.engine.end_step(loss)
        self._phase_open = False
        self._phase_loss = None
        return None if loss is None else float(loss)

    def train_epoch(self, dataloader, epoch: int) -> float:
        self._ensure_engine()
        self.current_epoch = epoch
        self.engine.epoch = epoch
        losses = []
        limit = self.config.batches_per_epoch
        skip, self.epoch_batch = self.epoch_batch, 0  # resumed mid-epoch: those batches are done
        for batch_idx, batch in enumerate(dataloader):
            if limit is not None and batch_idx >= limit:
                break
            if batch_idx < skip:
                self.epoch_batch = batch_idx + 1
                continue
            loss = self.engine.train_step(batch)
            self.epoch_batch = batch_idx + 1
            faults.maybe_inject(self.engine.rank, self.global_step, self.engine.heartbeat)
            if loss is not None:
                losses.append(loss)
            if self.engine.state_flags.get("under_attack") and self.training_state == TrainingState.TRAINING:
                self.training_state = TrainingState.UNDER_ATTACK
            if self.config.checkpoint_interval and self.global_step % self.config.checkpoint_interval == 0:
                self.save_checkpoint()
            if batch_idx % self.config.log_interval == 0 and loss is not None:
                logger.info("Epoch %d, Batch %d, Loss: %.4f", epoch, batch_idx, loss)
        last = self.engine.flush()
        if last is not None and (not losses or losses[-1] != last):
            losses.append(last)
        self.epoch_batch = 0
        self._sync_partitions()
        avg = float(np.mean(losses)) if losses else float("nan")
        logger.info("Epoch %d completed. Average loss: %.4f", epoch, avg)
        return avg

    def train(self, train_dataloader=None, val_dataloader=None, num_epochs: Optional[int] = None, *,
              dataset: Optional[str] = None, epochs: Optional[int] = None,
              trust_manager: Optional[TrustManager] = None):
        """Main loop (distributed_trainer.py:465-492) + README facade kwargs."""
        if trust_manager is not None and trust_manager is not self.trust_manager:
            trust_manager.resize(self.config.num_nodes)
            self.trust_manager = trust_manager
            if self.engine is not None:
                self.engine.trust = trust_manager
        if epochs is not None:
            num_epochs = epochs
        if num_epochs is None:
            num_epochs = self.config.num_epochs
        if train_dataloader is None:
            from ..utils.data_loader import get_dataloader
            name = dataset or self.config.dataset_name
            train_dataloader = get_dataloader(name, "train", self.config.batch_size, seq_len=self.config.seq_len,
                                              num_batches=self.config.batches_per_epoch or 10, seed=self.config.seed)
        self._ensure_engine()
        logger.info("Starting training for %d epochs", num_epochs)
        self.training_state = TrainingState.TRAINING
        history = []
        # a resumed job continues at the saved epoch (and, inside it, after the saved batch)
        for epoch in range(self.current_epoch, num_epochs):
            avg = self.train_epoch(train_dataloader, epoch)
            rec = {"epoch": epoch, "train_loss": avg}
            if val_dataloader is not None:
                rec["val_loss"] = self.validate(val_dataloader)
                logger.info("Validation loss: %.4f", rec["val_loss"])
            if self.training_state == TrainingState.UNDER_ATTACK:
                logger.info("Training under attack - implementing recovery measures")
                self.training_state = TrainingState.RECOVERING
                self.engine.state_flags["under_attack"] = False
            elif self.training_state == TrainingState.RECOVERING:
                self.training_state = TrainingState.TRAINING
            self.trust_manager.adaptive_threshold_adjustment()
            self.metrics_collector.collect_epoch_metrics(rec)
            history.append(rec)
        self.training_state = TrainingState.COMPLETED
        logger.info("Training completed successfully")
        return history

    def validate(self, val_dataloader, max_batches: Optional[int] = None) -> float:
        self._ensure_engine()
        total, n = 0.0, 0
        for i, batch in enumerate(val_dataloader):
            if max_batches is not None and i >= max_batches:
                break
            total += self.engine.eval_step(batch)
            n += 1
        return total / max(1, n)

    # ------------------------------------------------------------------ checkpointing
    def save_checkpoint(self, path: Optional[str] = None) -> str:
        from ..utils.checkpoint import save_checkpoint
        self._ensure_engine()
        return save_checkpoint(self, path)

    def load_checkpoint(self, path: str):
        from ..utils.checkpoint import load_checkpoint
        self._ensure_engine()
        load_checkpoint(self, path)
        self._sync_partitions()

    # ------------------------------------------------------------------ stats / teardown
    def get_training_stats(self) -> Dict:
        return {
            "current_epoch": self.current_epoch,
            "global_step": self.global_step,
            "training_state": self.training_state.value,
            "trust_scores": {i: self.trust_manager.get_trust_score(i) for i in range(self.config.num_nodes)},
            "attack_count": len(self.attack_history),
            "reassignment_count": len(self.reassignment_history),
            "metrics": self.metrics_collector.get_summary(),
            "plan": self.engine.plan.describe() if self.engine else None,
            "detection": self.attack_detector.get_detection_statistics(),
            "phase_ms": self.engine.tracer.summary() if self.engine and self.engine.tracer.enabled else {},
        }

    def cleanup(self):
        if self.engine is not None:
            self.engine.flush()
            self.engine.close()
        if self._owns_pg and dist.is_initialized():
            dist.destroy_process_group()
        logger.info("Distributed training cleanup completed")
