"""Configuration: reference-compatible dataclasses + the README YAML schema.

``TrainingConfig`` keeps every field of distributed_trainer.py:48-61 (same defaults) and adds
the engine knobs; ``load_config`` reads the README schema (README.md:111-132)::

    model: {name, size}
    training: {batch_size, learning_rate, num_epochs, seq_len, micro_batches, ...}
    distributed: {num_nodes, parallelism}
    security: {trust_threshold, attack_detection, gradient_verification, ...}
    attack: {enabled, types, target_nodes, intensity, start_step, ...}   (extension)

and the runner honours ``--config`` (the reference parses and ignores it: SURVEY A19).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, field, fields
from typing import Any, Dict, List, Optional

import yaml


@dataclass
class TrainingConfig:
    model_name: str = "gpt2"
    dataset_name: str = "openwebtext"
    batch_size: int = 32
    learning_rate: float = 5e-5
    num_epochs: int = 10
    num_nodes: int = 4
    trust_threshold: float = 0.7
    attack_detection_enabled: bool = True
    gradient_verification_enabled: bool = True
    checkpoint_interval: int = 100
    max_reassignment_attempts: int = 3
    # ---- extensions
    model_size: Optional[str] = None
    seq_len: int = 1024
    micro_batches: int = 4
    compute_dtype: str = "auto"
    weight_decay: float = 0.01
    max_grad_norm: float = 1.0
    adam_betas: List[float] = field(default_factory=lambda: [0.9, 0.999])
    checkpoint_dir: str = "checkpoints"
    reassignment_enabled: bool = True
    quarantine_enabled: bool = True
    trust_decay_per_step: float = 0.01
    parallelism: str = "model"           # "model" (pipeline) | "hybrid" (pipeline x data-parallel replicas)
    data_parallel: int = 1                # pipeline replicas (world size = stages x replicas)
    defer_wgrad: bool = True              # B/W split in the 1F1B schedule
    layer_granularity: str = "auto"       # pipeline units: "block" | "half" (GPT-2 attn/MLP) | "auto"
    num_classes: Optional[int] = None
    image_size: Optional[int] = None
    batches_per_epoch: Optional[int] = None
    log_interval: int = 10
    device: str = "auto"
    seed: int = 0
    verifier: Dict[str, Any] = field(default_factory=dict)
    heartbeat_interval: float = 0.0       # distributed: seconds between liveness beats (0 = off)
    heartbeat_timeout: float = 30.0       # silence after which a peer is OFFLINE
    abort_on_offline: bool = False        # exit non-zero on OFFLINE so an elastic restart resumes
                                          # from the latest checkpoint on the surviving ranks


@dataclass
class AttackSection:
    enabled: bool = False
    types: List[str] = field(default_factory=lambda: ["gradient_poisoning"])
    target_nodes: List[int] = field(default_factory=lambda: [1])
    intensity: float = 0.5
    start_step: int = 0
    end_step: Optional[int] = None
    probability: float = 1.0
    gradient_mode: str = "scale"


def _filter(cls, d: Dict[str, Any]) -> Dict[str, Any]:
    names = {f.name for f in fields(cls)}
    return {k: v for k, v in d.items() if k in names}


def load_config(path: str, overrides: Optional[Dict[str, Any]] = None):
    """Read a README-schema YAML file -> (TrainingConfig, AttackSection, raw dict)."""
    with open(path) as f:
        raw = yaml.safe_load(f) or {}
    tc: Dict[str, Any] = {}
    model = raw.get("model", {}) or {}
    if "name" in model:
        tc["model_name"] = model["name"]
    if "size" in model:
        tc["model_size"] = model["size"]
    for k in ("num_classes", "image_size"):
        if k in model:
            tc[k] = model[k]
    tr = raw.get("training", {}) or {}
    tc.update(_filter(TrainingConfig, tr))
    if "dataset" in tr:
        tc["dataset_name"] = tr["dataset"]
    if "dataset" in raw:
        tc["dataset_name"] = raw["dataset"] if isinstance(raw["dataset"], str) else raw["dataset"].get("name")
    ds = raw.get("distributed", {}) or {}
    if "num_nodes" in ds:
        tc["num_nodes"] = ds["num_nodes"]
    if "parallelism" in ds:
        tc["parallelism"] = ds["parallelism"]
    if "micro_batches" in ds:
        tc["micro_batches"] = ds["micro_batches"]
    if "data_parallel" in ds:
        tc["data_parallel"] = int(ds["data_parallel"])
    if "layer_granularity" in ds:
        tc["layer_granularity"] = str(ds["layer_granularity"])
    for k in ("heartbeat_interval", "heartbeat_timeout"):
        if k in ds:
            tc[k] = float(ds[k])
    if "abort_on_offline" in ds:
        tc["abort_on_offline"] = bool(ds["abort_on_offline"])
    sec = raw.get("security", {}) or {}
    mapping = {"trust_threshold": "trust_threshold", "attack_detection": "attack_detection_enabled",
               "gradient_verification": "gradient_verification_enabled", "reassignment": "reassignment_enabled",
               "quarantine": "quarantine_enabled", "max_reassignment_attempts": "max_reassignment_attempts",
               "trust_decay_per_step": "trust_decay_per_step"}
    for k, v in sec.items():
        if k in mapping:
            tc[mapping[k]] = v
    if "learning_rate" in tc:
        tc["learning_rate"] = float(tc["learning_rate"])  # YAML reads 5e-5 as a string
    if overrides:
        tc.update({k: v for k, v in overrides.items() if v is not None})
    atk = AttackSection(**_filter(AttackSection, raw.get("attack", {}) or {}))
    return TrainingConfig(**_filter(TrainingConfig, tc)), atk, raw


def dump_config(cfg: TrainingConfig, attack: Optional[AttackSection], path: str):
    d = asdict(cfg)
    out = {
        "model": {"name": d.pop("model_name"), "size": d.pop("model_size")},
        "training": {k: d.pop(k) for k in ("batch_size", "learning_rate", "num_epochs", "seq_len",
                                           "micro_batches", "dataset_name")},
        "distributed": {"num_nodes": d.pop("num_nodes"), "parallelism": d.pop("parallelism"),
                        "data_parallel": d.pop("data_parallel"),
                        "layer_granularity": d.pop("layer_granularity")},
        "security": {"trust_threshold": d.pop("trust_threshold"),
                     "attack_detection": d.pop("attack_detection_enabled"),
                     "gradient_verification": d.pop("gradient_verification_enabled")},
        "extra": d,
    }
    if attack is not None:
        out["attack"] = asdict(attack)
    with open(path, "w") as f:
        yaml.safe_dump(out, f, sort_keys=False)
