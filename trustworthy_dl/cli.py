"""``trustworthy-dl-train`` console entry point (setup_py.py:63; phantom ``cli.main`` in the reference).

    trustworthy-dl-train --config configs/gpt2_distributed.yaml [--epochs N] [--nodes N] ...
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m trustworthy_dl.cli --config ...

Single process: the local backend simulates ``num_nodes`` stages (spread over the visible GPUs).
Under torchrun (WORLD_SIZE > 1): one stage per rank over RCCL (GPU) / gloo (CPU).
"""
from __future__ import annotations

import argparse
import json
import logging
import os
import sys


def main(argv=None):
    p = argparse.ArgumentParser(description="trustworthy model-parallel training")
    p.add_argument("--config", type=str, default=None)
    p.add_argument("--model", type=str, default=None)
    p.add_argument("--size", type=str, default=None)
    p.add_argument("--dataset", type=str, default=None)
    p.add_argument("--nodes", type=int, default=None)
    p.add_argument("--epochs", type=int, default=None)
    p.add_argument("--batch-size", type=int, default=None)
    p.add_argument("--lr", type=float, default=None)
    p.add_argument("--seq-len", type=int, default=None)
    p.add_argument("--micro-batches", type=int, default=None)
    p.add_argument("--batches-per-epoch", type=int, default=None)
    p.add_argument("--checkpoint-dir", type=str, default=None)
    p.add_argument("--resume", type=str, default=None, help="checkpoint path or 'latest'")
    p.add_argument("--attack", action="store_true")
    p.add_argument("--device", type=str, default=None)
    p.add_argument("--heartbeat", type=float, default=None, help="seconds between liveness beats (0 = off)")
    p.add_argument("--heartbeat-timeout", type=float, default=None, help="silence (s) after which a peer is OFFLINE")
    p.add_argument("--checkpoint-interval", type=int, default=None, help="optimizer steps between checkpoints")
    p.add_argument("--dtype", type=str, default=None, choices=["bf16", "fp32"], help="compute dtype")
    p.add_argument("--abort-on-offline", action="store_true",
                   help="exit non-zero when a peer goes OFFLINE; restart the job with --resume latest "
                        "on the surviving ranks (the checkpoint is re-planned over them)")
    a = p.parse_args(argv)
    logging.basicConfig(level=logging.INFO)

    from .attacks import AdversarialAttacker, AttackConfig
    from .config import AttackSection, TrainingConfig, load_config
    from .core.distributed_trainer import DistributedTrainer
    from .utils.checkpoint import latest_checkpoint

    over = {"model_name": a.model, "model_size": a.size, "dataset_name": a.dataset, "num_nodes": a.nodes,
            "num_epochs": a.epochs, "batch_size": a.batch_size, "learning_rate": a.lr, "seq_len": a.seq_len,
            "micro_batches": a.micro_batches, "batches_per_epoch": a.batches_per_epoch,
            "checkpoint_dir": a.checkpoint_dir, "device": a.device, "heartbeat_interval": a.heartbeat,
            "heartbeat_timeout": a.heartbeat_timeout, "checkpoint_interval": a.checkpoint_interval,
            "compute_dtype": a.dtype,
            "abort_on_offline": True if a.abort_on_offline else None}
    if a.config:
        cfg, atk, _ = load_config(a.config, over)
    else:
        cfg = TrainingConfig(**{k: v for k, v in over.items() if v is not None})
        atk = AttackSection()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    attacker = None
    if a.attack or atk.enabled:
        attacker = AdversarialAttacker(AttackConfig(attack_types=atk.types, target_nodes=atk.target_nodes,
                                                    intensity=atk.intensity, start_step=atk.start_step,
                                                    end_step=atk.end_step, probability=atk.probability,
                                                    gradient_mode=atk.gradient_mode))
        attacker.activate_attacks()
    trainer = DistributedTrainer(cfg, attacker=attacker)
    if world > 1:
        trainer.setup_distributed_environment(int(os.environ["RANK"]), world)
    trainer.create_model_partitions()
    if a.resume:
        path = latest_checkpoint(cfg.checkpoint_dir) if a.resume == "latest" else a.resume
        if path:
            trainer.load_checkpoint(path)
    trainer.train()
    stats = trainer.get_training_stats()
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps(stats, indent=2, default=str))
    trainer.cleanup()
    return stats


if __name__ == "__main__":
    sys.exit(0 if main() is not None else 1)
