"""Configuration of the pipeline engine (parallel/pipeline.py): the reference's TrainingConfig
knobs (distributed_trainer.py:48-61) extended with the micro-batch schedule, verification, audit,
re-shard and communication settings."""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional

import torch

from .flat import AdamWConfig


@dataclass
class EngineConfig:
    num_nodes: int = 1                  # local mode: logical stages; distributed: world size
    micro_batches: int = 1
    compute_dtype: str = "auto"          # auto -> bf16 on GPU, fp32 on CPU
    device: str = "auto"
    balanced_partition: bool = True
    seq_len: Optional[int] = None        # for GPT cost model
    adamw: AdamWConfig = field(default_factory=AdamWConfig)
    attack_detection: bool = True        # output anomaly detection
    gradient_verification: bool = True
    quarantine: bool = True              # skip flagged gradient updates on device
    verifier: Dict[str, Any] = field(default_factory=dict)
    trust_threshold: float = 0.7
    trust_decay_per_step: float = 0.01
    reassign: bool = True
    max_reassignment_attempts: int = 3
    output_check: str = "random"         # which micro-batch output is monitored each step: "random" (a
                                         # per-step choice from a private seeded RNG, so an attacker
                                         # cannot predict which output is inspected) | "first" | "none"
    monitor_seed: Optional[int] = None   # seed of that RNG (None: $TDL_MONITOR_SEED, else os.urandom)
    early_grad_stats: bool = True        # start each layer's gradient statistics on the side stream
                                         # as soon as its last-micro-batch backward is done
    defer_wgrad: bool = True             # B/W split: weight grads run after dx is posted upstream
    data_parallel: int = 1               # pipeline replicas (distributed): world = stages x replicas
    param_audit_interval: int = 10       # DP: steps between cross-replica weight-digest audits (0 = off)
    param_integrity: bool = True         # checksum compute weights after each update, re-check before the next
    shadow_interval: int = 25            # steps between trusted weight snapshots held by the next stage's GPU
                                         # (0 = off); a compromised stage is restored from it, not from itself.
                                         # A snapshot is also taken when the stages are (re)built
    audit: bool = True                   # deterministic stage cross-check: the next stage recomputes every
                                         # non-loss stage's monitored micro-batch from its input and weights and
                                         # compares the output it received; blame for a tampered forward comes
                                         # only from such a mismatch or a failed weight-integrity check, output
                                         # z-scores no longer blame (they stay in the trust metrics)
    audit_prob: float = 1.0              # fraction of steps audited (drawn privately by each auditor)
    audit_backward: bool = True          # the audit covers the backward too: the auditor recomputes the
                                         # audited micro-batch's input gradient and the sketch of its
                                         # weight-gradient contribution (security/grad_audit.py), the
                                         # loss stage is audited by its predecessor, and every stage's
                                         # applied gradient must equal the sum of its committed
                                         # per-micro-batch contributions; gradient z-scores then no longer
                                         # blame (they quarantine the update and feed the trust metrics)
    audit_grad_tol: float = 0.05         # relative keyed-sketch error above which a gradient check fails
    audit_micro_k: int = 1               # micro-batches audited per audited step and stage (k of M, drawn
                                         # privately and uniformly; a tamper of one micro-batch is caught
                                         # with probability k / M per step, 1 - (1 - k/M)^s within s steps)
    audit_targeted: Optional[bool] = None  # besides the private uniform choice, also audit the micro-batch
                                         # whose output statistics (log RMS, sign of the token-mean vector)
                                         # or committed gradient-sketch norm stand out among the step's M
                                         # (robust z > audit_target_z): a one-of-M tamper that moves them is
                                         # then recomputed in the step it happens, not with probability 1/M.
                                         # None = local mode only (distributed: one device->host read of the
                                         # M scores per auditor and step, opt-in with True)
    layer_granularity: str = "auto"      # "block" | "half" (GPT-2 attention / MLP halves as pipeline
                                         # units) | "auto": half when it lowers the slowest stage
    p2p_mode: str = "async"              # "async": per-direction communicators + receives posted a phase
                                         # ahead; "grouped": one batch_isend_irecv per exchange
    heartbeat_interval: float = 0.0      # distributed: seconds between heartbeats (0 = watchdog off)
    heartbeat_timeout: float = 30.0      # silence after which a peer is OFFLINE
    abort_on_offline: bool = False       # fail fast so an elastic launcher restarts from a checkpoint
    seed: int = 0
    trace_phases: bool = False           # HIP-event per-phase step breakdown (runtime/tracing.py)
    serialize_streams: bool = field(default_factory=lambda: os.environ.get("TDL_SERIALIZE_STREAMS", "0") == "1")
                                         # debug: verification on the compute stream (no side-stream overlap)

    # ---- fixed policy constants: class attributes, not constructor knobs (no test, record or
    # experiment varies them; read as cfg.<name> like the fields above)
    min_stages = 1
    compromise_after = 2        # consecutive flagged steps before mark_compromised (1 = reference)
    robust_aggregation = True   # DP: flagged / outlier replicas are left out of the gradient mean
    outlier_ratio = 4.0         # DP (>= 3 replicas): grad norm vs replica median beyond this = outlier
    direction_margin = 0.2      # DP (>= 3 replicas): cosine to the other replicas' sum below 0 and
                                # this far below the median = outlier (sign flips)
    shadow_copies = 2           # holders per snapshot (the next 1-2 stages of the ring): a stage
                                # whose first holder is compromised too is still restorable
    audit_tol = 1e-2            # relative max error above which a recomputed output mismatches
    audit_target_z = 4.0        # robust z of a micro-batch score that makes the targeted audit pick it
    compromise_on_proof = True  # a failed audit / integrity / gradient-consistency check (proof of
                                # tampering, not a statistic) compromises the node at once
    attribute_flags = True      # blame the earliest anomalous stage, not its downstream/upstream echoes
    soft_output_z = 5.0         # with an output flag in a replica, an EARLIER stage whose output z
                                # exceeds this (below its own decision threshold) is the source
    global_event_fraction = 0.5  # gradient anomalies on >= this fraction of a replica's stages (>= 3)
                                 # in one step = a pipeline-wide event (a loss spike of real training):
                                 # the update is skipped, nobody is blamed, and blame stays off for
                                 # ``global_event_grace`` steps while the detector baselines re-settle
    global_event_grace = 8
    pipeline_quarantine = True  # output / integrity evidence anywhere skips the whole replica's update


def _resolve_dtype(name: str, device: torch.device) -> torch.dtype:
    if name == "auto":
        return torch.bfloat16 if device.type == "cuda" else torch.float32
    return {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp32": torch.float32,
            "float32": torch.float32}[name]


def split_micro(t: torch.Tensor, m: int) -> List[torch.Tensor]:
    if t.shape[0] % m != 0:
        raise ValueError(f"batch {t.shape[0]} not divisible by micro_batches {m}")
    return list(t.chunk(m, dim=0))
