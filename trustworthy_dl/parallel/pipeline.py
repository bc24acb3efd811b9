"""Trust-aware pipeline-parallel training engine.

Two execution modes share every component (stages, flat buffers, verifiers, trust kernels):

* ``distributed`` — one process per GPU (``torch.distributed``: RCCL on MI355X, gloo on CPU).
  Each rank runs one stage with a 1F1B schedule over M micro-batches; activations and their
  gradients cross stage boundaries as grouped P2P over xGMI.  This makes the reference's
  logical "nodes" (distributed_trainer.py:148-207 — all partitions in one process, sequential,
  no P2P) real pipeline stages.
* ``local`` — all stages in one process (optionally spread over the visible devices); the
  deterministic simulation backend used for fault-injection tests.

Per step and per stage: forward/backward over micro-batches -> tied-embedding gradient all-reduce
(first<->last stage) -> device verification (stage_verifier.py) -> all-gather of the per-stage
digest rows -> fused trust update on every rank (identical inputs => identical decisions) ->
fused AdamW that skips quarantined gradients on device.  The host reads the step report one step
later (pinned, non-blocking) to update TrustManager / AttackDetector mirrors, histories and to
trigger task reassignment (re-shard over the trusted set) — the same decision on every rank.
"""
from __future__ import annotations

import copy
import logging
import math
import os
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from ..core.trust_manager import (METRIC_NAMES, NodeStatus, STATUS_CODES, STATUS_FROM_CODE, TrustManager)
from ..security import stage_verifier as SV
from ..ops import stats as dstats
from ..ops.layers import bump_weight_generation
from ..ops.layers import defer_weight_grads
from ..runtime.commcheck import note_host_sync
from ..runtime.tracing import PhaseTracer
from . import comm as p2p
from .comm import LinkMeter, P2PComm, all_gather_rows, batched_transfer, broadcast_ints
from .flat import AdamWConfig
from .partition import PlacementPlan, make_plan
from .stage import Stage, tied_groups
from ..runtime import progress

logger = logging.getLogger(__name__)


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
    min_stages: int = 1
    output_check: str = "random"         # which micro-batch output is monitored each step: "random" (a
                                         # per-step choice from a private seeded RNG, so an attacker
                                         # cannot predict which output is inspected) | "first" | "none"
    monitor_seed: Optional[int] = None   # seed of that RNG (None: $TDL_MONITOR_SEED, else os.urandom)
    early_grad_stats: bool = True        # start each layer's gradient statistics on the side stream
                                         # as soon as its last-micro-batch backward is done
    compromise_after: int = 2            # consecutive flagged steps before mark_compromised (1 = reference)
    defer_wgrad: bool = True             # B/W split: weight grads run after dx is posted upstream
    data_parallel: int = 1               # pipeline replicas (distributed): world = stages x replicas
    robust_aggregation: bool = True      # DP: flagged / outlier replicas are left out of the gradient mean
    outlier_ratio: float = 4.0           # DP (>= 3 replicas): grad norm vs replica median beyond this = outlier
    direction_margin: float = 0.2        # DP (>= 3 replicas): cosine to the other replicas' sum below 0 and
                                         # this far below the median = outlier (sign flips)
    param_audit_interval: int = 10       # DP: steps between cross-replica weight-digest audits (0 = off)
    param_integrity: bool = True         # checksum compute weights after each update, re-check before the next
    shadow_interval: int = 25            # steps between trusted weight snapshots held by the next stage's GPU
                                         # (0 = off); a compromised stage is restored from it, not from itself.
                                         # A snapshot is also taken when the stages are (re)built
    shadow_copies: int = 2               # holders per snapshot (the next 1-2 stages of the ring): a stage
                                         # whose first holder is compromised too is still restorable
    audit: bool = True                   # deterministic stage cross-check: the next stage recomputes every
                                         # non-loss stage's monitored micro-batch from its input and weights and
                                         # compares the output it received; blame for a tampered forward comes
                                         # only from such a mismatch or a failed weight-integrity check, output
                                         # z-scores no longer blame (they stay in the trust metrics)
    audit_prob: float = 1.0              # fraction of steps audited (drawn privately by each auditor)
    audit_tol: float = 1e-2              # relative max error above which a recomputed output mismatches
    audit_backward: bool = True          # the audit covers the backward too: the auditor recomputes the
                                         # audited micro-batch's input gradient and the sketch of its
                                         # weight-gradient contribution (security/grad_audit.py), the
                                         # loss stage is audited by its predecessor, and every stage's
                                         # applied gradient must equal the sum of its committed
                                         # per-micro-batch contributions; gradient z-scores then no longer
                                         # blame (they quarantine the update and feed the trust metrics)
    audit_grad_tol: float = 0.05         # relative sketch error above which a gradient check fails
    audit_targeted: Optional[bool] = None  # besides the private uniform choice, also audit the micro-batch
                                         # whose output statistics (log RMS, sign of the token-mean vector)
                                         # or committed gradient-sketch norm stand out among the step's M
                                         # (robust z > audit_target_z): a one-of-M tamper that moves them is
                                         # then recomputed in the step it happens, not with probability 1/M.
                                         # None = local mode only (distributed: one device->host read of the
                                         # M scores per auditor and step, opt-in with True)
    audit_target_z: float = 4.0
    compromise_on_proof: bool = True     # a failed audit / integrity / gradient-consistency check (proof of
                                         # tampering, not a statistic) compromises the node at once
    attribute_flags: bool = True         # blame the earliest anomalous stage, not its downstream/upstream echoes
    soft_output_z: float = 5.0           # with an output flag in a replica, an EARLIER stage whose output z
                                         # exceeds this (below its own decision threshold) is the source: a
                                         # tampered output moves its own statistics at least as much as the
                                         # downstream echoes (0 = off)
    global_event_fraction: float = 0.5   # gradient anomalies on >= this fraction of a replica's stages (>= 3
                                         # stages) in one step = a pipeline-wide event (a loss spike of real
                                         # training), not a Byzantine stage: the step's update is skipped, nobody
                                         # is blamed, and blame stays off for ``global_event_grace`` steps while
                                         # the detector baselines re-settle
    global_event_grace: int = 8
    pipeline_quarantine: bool = True     # output / integrity evidence anywhere skips the whole replica's update
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


def _resolve_dtype(name: str, device: torch.device) -> torch.dtype:
    if name == "auto":
        return torch.bfloat16 if device.type == "cuda" else torch.float32
    return {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp32": torch.float32,
            "float32": torch.float32}[name]


def split_micro(t: torch.Tensor, m: int) -> List[torch.Tensor]:
    if t.shape[0] % m != 0:
        raise ValueError(f"batch {t.shape[0]} not divisible by micro_batches {m}")
    return list(t.chunk(m, dim=0))


class PipelineEngine:
    def __init__(self, model: nn.Module, cfg: EngineConfig, trust_manager: Optional[TrustManager] = None,
                 attacker=None, metrics=None, detector=None):
        self.cfg = cfg
        self.model = model                       # CPU master copy: layer skeletons for (re)sharding
        self.distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self.rank = dist.get_rank() if self.distributed else 0
        self.world = dist.get_world_size() if self.distributed else 1
        self.num_nodes = self.world if self.distributed else cfg.num_nodes
        # data parallelism over pipeline replicas: rank = replica * pp + stage position
        self.dp = max(1, int(cfg.data_parallel)) if self.distributed else 1
        if self.world % self.dp:
            raise ValueError(f"world size {self.world} not divisible by data_parallel={self.dp}")
        self.pp = self.world // self.dp if self.distributed else cfg.num_nodes
        self.replica = self.rank // self.pp if self.distributed else 0
        self.dp_group = None
        self.dp_audits: List[Dict] = []
        self.trust = trust_manager or TrustManager(self.num_nodes, cfg.trust_threshold)
        self.trust.resize(self.num_nodes)
        self.attacker = attacker
        self.metrics = metrics
        self.detector = detector
        self.global_step = 0
        self.epoch = 0
        self.attack_history: List[Dict] = []
        self.reassignment_history: List[Dict] = []
        self.excluded: List[int] = []
        self.state_flags = {"under_attack": False}
        self.p2p_mode = self._choose_p2p_mode(cfg)
        self.granularity = self._choose_granularity(model, cfg)
        self.layers = model.pipeline_layers()
        self.num_layers = len(self.layers)
        self.ties = tied_groups(model)
        self.last_loss: Optional[float] = None
        self._pending: deque = deque()
        self._reset_shadows()
        self._host_metrics: Dict[int, List[float]] = {}
        self._comm_wait = 0.0
        self._step_time = 0.0
        # private per-process RNG for the monitored micro-batch (not derived from the data seed)
        seed = cfg.monitor_seed
        if seed is None and os.environ.get("TDL_MONITOR_SEED"):
            seed = int(os.environ["TDL_MONITOR_SEED"])   # reproducible runs / tests
        if seed is None:
            seed = int.from_bytes(os.urandom(8), "little")
        self._mon_rng = __import__("random").Random(seed)
        self._mon_idx = 0
        self._targeted = False

        if cfg.device == "auto":
            if torch.cuda.is_available():
                lr = int(os.environ.get("LOCAL_RANK", self.rank % max(1, torch.cuda.device_count())))
                self.device = torch.device("cuda", lr % torch.cuda.device_count())
            else:
                self.device = torch.device("cpu")
        else:
            self.device = torch.device(cfg.device)
        if self.device.type == "cuda":
            torch.cuda.set_device(self.device)
        # conv nets run bf16 on the native NHWC implicit-GEMM kernels (ops/conv.py), like GPT-2
        self.dtype = _resolve_dtype(cfg.compute_dtype, self.device)
        self.tracer = PhaseTracer(self.device, enabled=cfg.trace_phases)

        self.costs = self._model_costs(model, cfg)
        n_stages = min(self.pp, self.num_layers)
        base = self.replica * self.pp
        self.plan = make_plan(self.costs, [base + i for i in range(n_stages)], 0, cfg.balanced_partition)
        self._init_trust_state()
        self._build()
        self._init_build_times = dict(self._build_times)
        self.link_meter = LinkMeter(150e9 if self.device.type == "cuda" else 2e9)
        self.heartbeat = None
        self.node_events: List[Dict] = []
        self.quarantine_on_evidence = cfg.quarantine and cfg.pipeline_quarantine
        if self.distributed and cfg.heartbeat_interval > 0:
            from ..runtime.heartbeat import HeartbeatMonitor
            store = dist.distributed_c10d._get_default_store()
            self.heartbeat = HeartbeatMonitor(store, self.rank, self.world, cfg.heartbeat_interval,
                                              cfg.heartbeat_timeout, abort_on_offline=cfg.abort_on_offline).start()
        self.refresh_shadows()   # a committed trusted copy of every stage from step 0 on
        logger.info("PipelineEngine[%s] plan: %s", "dist" if self.distributed else "local", self.plan.describe())

    # ================================================================== construction
    def _model_costs(self, model: nn.Module, cfg: EngineConfig) -> List[float]:
        if hasattr(model, "config") and hasattr(model, "layer_costs") and getattr(model, "family", "") == "gpt2":
            return model.layer_costs(cfg.seq_len or model.config.n_positions)
        if hasattr(model, "layer_costs"):
            return model.layer_costs()
        return [1.0] * len(model.pipeline_layers())

    def _choose_granularity(self, model: nn.Module, cfg: EngineConfig) -> str:
        """Pick the pipeline unit size for models that offer several (GPT-2 blocks or halves):
        ``auto`` takes half blocks only when that lowers the slowest stage's cost by > 2%."""
        if not hasattr(model, "set_pipeline_granularity"):
            return "block"
        want = cfg.layer_granularity
        if want == "auto":
            best = {}
            for g in ("block", "half"):
                model.set_pipeline_granularity(g)
                costs = self._model_costs(model, cfg)
                n = min(self.pp, len(costs))
                rngs = make_plan(costs, list(range(n)), 0, cfg.balanced_partition).ranges
                best[g] = max(sum(costs[a:b]) for a, b in rngs)
            want = "half" if best["half"] < 0.98 * best["block"] else "block"
        model.set_pipeline_granularity(want)
        return want

    def set_granularity(self, granularity: str) -> None:
        """Switch the pipeline unit size (e.g. to match a checkpoint); the caller then installs a
        plan over the new unit list and rebuilds (stage weights are reloaded by the caller)."""
        if not hasattr(self.model, "set_pipeline_granularity"):
            if granularity != "block":
                raise ValueError(f"{type(self.model).__name__} has only whole-layer pipeline units")
            return
        self.model.set_pipeline_granularity(granularity)
        self.granularity = granularity
        self.layers = self.model.pipeline_layers()
        self.num_layers = len(self.layers)
        self.ties = tied_groups(self.model)
        self.costs = self._model_costs(self.model, self.cfg)

    def _stage_device(self, node: int) -> torch.device:
        if self.distributed or self.device.type != "cuda":
            return self.device
        n = torch.cuda.device_count()
        return torch.device("cuda", node % n)

    def _verifier_kwargs(self) -> dict:
        vk = dict(self.cfg.verifier)
        vk.setdefault("quarantine", self.cfg.quarantine)
        vk.setdefault("output_detection", self.cfg.attack_detection)
        vk.setdefault("gradient_verification", self.cfg.gradient_verification)
        vk.setdefault("serialize_streams", self.cfg.serialize_streams)
        # a verifier built by a re-plan (re-shard, resume) warms its baselines while attacks may be
        # running: gross outliers are flagged and kept out of the baseline from its 8th entry on.
        # The first build warms up on the start of training, which is assumed clean (as the
        # reference's warm-up does) and whose early transients must not be flagged.
        vk.setdefault("early_gate", getattr(self, "_built_once", False))
        return vk

    def _build(self, layer_modules: Optional[Dict[int, nn.Module]] = None):
        """Build this rank's stages of the current plan.  ``layer_modules`` (re-shard): layer index
        -> a module this rank already holds on a device; those are re-used (re-bound to the new
        stage's flat buffers), every other layer is deep-copied from the host model and moved to
        the device.  The two costs are timed separately (``_build_times``): they calibrate the
        rebuild term of ``estimate_migration_time``."""
        self._sync_all()
        t0 = time.perf_counter()
        built = []
        fresh = 0
        for sid, (node, rng) in enumerate(zip(self.plan.ranks, self.plan.ranges)):
            if self.distributed and node != self.rank:
                continue
            a, b = rng
            layers = []
            memo: Dict[int, Any] = {}   # one memo per stage: parameters tied inside it stay shared
            for li in range(a, b):
                m = layer_modules.get(li) if layer_modules else None
                if m is None:
                    m = copy.deepcopy(self.layers[li], memo)
                    fresh += self._layer_numel(li)
                layers.append(m)
            if layer_modules:
                self._retie(layers, a, b)
            dev = self._stage_device(node)
            layers = [m.to(dev) for m in layers]
            built.append((sid, node, rng, layers, dev))
        self._sync_all()
        t1 = time.perf_counter()
        self.stages: Dict[int, Stage] = {}
        total = 0
        for sid, node, rng, layers, dev in built:
            st = Stage(self.model, rng, sid, self.plan.num_stages, dev, self.dtype, self._verifier_kwargs(),
                       layers=layers)
            total += st.flat.numel
            self.stages[node] = st
        self._set_clip_exclusions()
        self._set_early_stats()
        self._sync_all()
        t2 = time.perf_counter()
        self._build_comm()
        t3 = time.perf_counter()
        self._built_once = True
        self._build_times = {"materialize_s": t1 - t0, "materialized_params": fresh, "flatten_s": t2 - t1,
                             "flattened_params": total, "stages": len(built), "groups_s": t3 - t2}

    def _sync_all(self):
        note_host_sync(device=True)
        if self.device.type == "cuda":
            torch.cuda.synchronize()

    def _retie(self, layers: List[nn.Module], a: int, b: int):
        """Re-used layer modules may come from different old stages (or share a tied parameter with a
        layer that now lives on another stage): every tie group's members inside [a, b) get one
        fresh, stage-private parameter (its value is overwritten by the migrated master weights)."""
        for grp in self.ties:
            members = [(li, attr) for li, attr in grp if a <= li < b]
            if not members:
                continue
            src = layers[members[0][0] - a]
            *path, leaf = members[0][1].split(".")
            for part in path:
                src = getattr(src, part)
            old = getattr(src, leaf)
            fresh = nn.Parameter(old.detach().clone(), requires_grad=old.requires_grad)
            for li, attr in members:
                obj = layers[li - a]
                *path, leaf = attr.split(".")
                for part in path:
                    obj = getattr(obj, part)
                setattr(obj, leaf, fresh)

    def _set_early_stats(self):
        """Per-layer gradient-statistics triggers (verification overlapped with the backward).
        Tied weights are reduced across stages after the backward and simulated gradient attacks
        rewrite the flat gradient after it: both stay with the final pass."""
        if not self.cfg.early_grad_stats or (self.attacker is not None and hasattr(self.attacker, "on_gradients")):
            return
        # only where every parameter gradient is written by the layer's own backward into
        # main_grad (the GPT-2 fused ops): a torch module's .grad is folded in by a separate
        # accumulate hook whose order against the input-gradient hook is not fixed
        if getattr(self.model, "family", "") != "gpt2" or self.device.type != "cuda":
            return
        tied = set()
        for grp in self.ties:
            for node, st in self.stages.items():
                for li, attr in grp:
                    prm = st.local_param(li, attr)
                    if prm is not None:
                        tied.add(id(prm))
        for st in self.stages.values():
            st.set_early_stats(tied)
            # early tied all-reduce only with hardware queues to spare (the p2p "async" mode): its
            # RCCL kernel waits on a stream of its own for the embedding stage, and on a queue
            # shared with the compute stream it would block the rest of this stage's backward
            st.on_tied_ready = (self._launch_tied_allreduce
                                if self.distributed and self.p2p_mode == "async" and len(self.ties) == 1 else None)

    def _set_clip_exclusions(self):
        """Count every tied weight once in the global clipping norm: the stage owning the first
        member of a tie group (the embedding) counts it, other stages' copies are excluded."""
        for node, st in self.stages.items():
            ex = set()
            for grp in self.ties:
                if self.plan.owner_of_layer(grp[0][0]) == node:
                    continue
                for li, attr in grp:
                    prm = st.local_param(li, attr)
                    if prm is not None:
                        ex.add(id(prm))
            st.set_clip_exclusions(ex)

    def _build_comm(self):
        """Communicators and streams of one rank (every one of them, by purpose):

        * default group (init_process_group): digest all-gather, plan broadcast, clip-norm / step
          all-reduces, migration and shadow-snapshot P2P (RCCL creates one 2-rank communicator per
          peer pair it sends to or receives from);
        * ``_dir_groups`` (async P2P mode): one group for activations (stage s -> s+1) and one for
          activation gradients (s+1 -> s), each with a 2-rank communicator per neighbour pair;
        * tie group (tied embedding / LM head on different ranks): the tied-gradient all-reduce;
        * DP group (data_parallel > 1): the replica gradient all-reduce and direction check.
        Under torch's RCCL backend every communicator has one stream of its own; add the compute
        stream and one verification side stream per local stage (security/stage_verifier.py).
        Groups are cached by member set and reused across re-plans (a re-shard creates a group only
        for a member set never seen before; ``comm_inventory`` reports the totals against the
        hardware-queue budget, runtime/hwqueues.py)."""
        self.comm = None
        self.tie_group = None
        self.tie_members: List[int] = []
        if not hasattr(self, "_group_cache"):
            self._group_cache: Dict[Tuple[str, Tuple[int, ...]], object] = {}
            self._p2p_peers: Dict[str, set] = {}
        if not self.distributed:
            return
        s = self.plan.stage_of_rank(self.rank)
        prev = self.plan.ranks[s - 1] if s is not None and s > 0 else None
        nxt = self.plan.ranks[s + 1] if s is not None and s + 1 < self.plan.num_stages else None
        self.comm = P2PComm(prev, nxt, self.device)
        for peer in (prev, nxt):
            if peer is not None:
                self._p2p_peers.setdefault("default" if self.p2p_mode != "async" else "dir", set()).add(peer)
        if self.p2p_mode == "async" and getattr(self, "_dir_groups", None) is None:
            # one communicator for activations (stage s -> s+1), one for activation gradients
            # (s+1 -> s): each carries one-way, in-order traffic per neighbour pair
            everyone = list(range(self.world))
            self._dir_groups = (self._group("act", everyone), self._group("grad", everyone))
        if self.cfg.audit and getattr(self, "_audit_pg", None) is None:
            # the audit's weight shipment runs on its own communicator, posted before the schedule
            # and overlapped with it (``_audit_early_ship``)
            self._audit_pg = self._group("audit", list(range(self.world)))
        # tied parameters living on different ranks need a gradient all-reduce group (one per
        # replica; new_group is collective over the whole world, so every rank creates them all)
        base = self.replica * self.pp
        local = sorted({self.plan.owner_of_layer(li) - base for grp in self.ties for li, _ in grp})
        self.tie_members = [base + r for r in local] if len(local) > 1 else []
        if len(local) > 1:
            for d in range(self.dp):
                g = self._group("tie", [d * self.pp + r for r in local])
                if d == self.replica:
                    self.tie_group = g
        if self.dp > 1 and self.dp_group is None:
            for pos in range(self.pp):
                g = self._group("dp", [d * self.pp + pos for d in range(self.dp)])
                if pos == self.rank % self.pp:
                    self.dp_group = g

    def _group(self, purpose: str, members: List[int]):
        """The process group of ``members`` for ``purpose``, created (collectively, in the same
        order on every rank) and warmed only the first time this member set is asked for."""
        key = (purpose, tuple(members))
        g = self._group_cache.get(key)
        if g is None:
            g = dist.new_group(ranks=list(members))
            self._warm_group(g, list(members))
            self._group_cache[key] = g
        return g

    def _note_peers(self, sends, recvs, kind: str = "default"):
        peers = getattr(self, "_p2p_peers", None)
        if peers is not None:
            peers.setdefault(kind, set()).update(int(p) for _, p in list(sends) + list(recvs))

    def comm_inventory(self) -> Dict[str, object]:
        """Per-rank communicator / stream count by purpose, against the HIP hardware-queue budget.
        Communicators: the default group's, one per cached group this rank belongs to, and one
        2-rank P2P communicator per (group, peer) this rank has exchanged with."""
        groups = [{"purpose": p, "members": list(m)} for (p, m) in getattr(self, "_group_cache", {})]
        mine = [g for g in groups if self.rank in g["members"]]
        p2p = {k: sorted(v) for k, v in getattr(self, "_p2p_peers", {}).items()}
        n_p2p = sum(len(v) * (2 if k == "dir" else 1) for k, v in p2p.items())
        n_comms = (1 if self.distributed else 0) + len(mine) + n_p2p
        streams = 1 + len(self.stages) + n_comms   # compute + verification side streams + RCCL streams
        from ..runtime.hwqueues import effective_hw_queues
        q = effective_hw_queues() if self.device.type == "cuda" else None
        return {"groups_created": len(groups), "groups_member": len(mine), "p2p_peers": p2p,
                "rccl_comms": n_comms, "hip_streams": streams, "hw_queues": q,
                "within_queue_budget": q is None or streams <= q}

    def _choose_p2p_mode(self, cfg: EngineConfig) -> str:
        """Pre-posted receives ("async") need the RCCL streams on hardware queues of their own:
        an RCCL receive spins until its data lands, and a compute kernel queued behind it on a shared
        queue cannot run (runtime/hwqueues.py, profiles/r1_hwqueue_probe.json).  When the HIP runtime
        started with too few queues (GPU touched before ``trustworthy_dl`` was imported, or
        TDL_KEEP_HW_QUEUES=1), fall back to grouped exchanges, which post a receive only where the
        compute needs its data anyway."""
        mode = cfg.p2p_mode
        if mode == "async" and self.distributed and dist.get_backend() == "nccl":
            from ..runtime.hwqueues import ENGINE_QUEUES, effective_hw_queues
            q = effective_hw_queues()
            if q < ENGINE_QUEUES:
                logger.warning("GPU_MAX_HW_QUEUES=%d < %d: pipeline P2P falls back to grouped exchanges",
                               q, ENGINE_QUEUES)
                mode = "grouped"
        return mode

    def _warm_group(self, group, members: List[int]):
        """One 1-element all-reduce by every member, right after the group is created (groups are
        created in the same order on every rank, so members meet in that order).  Under RCCL this
        brings the communicator up collectively before the first pipeline P2P on it, which is posted
        by only a subset of the ranks (torch's batch_isend_irecv requirement for the first call on a
        group); under gloo it is a cheap rendezvous check."""
        if self.rank not in members or len(members) < 2:
            return
        t = torch.zeros(1, device=self.device)
        dist.all_reduce(t, group=group)

    def _init_trust_state(self):
        N = self.num_nodes
        dev = self.device
        self.t_values = torch.tensor([self.trust.get_trust_score(i) for i in range(N)], dtype=torch.float32, device=dev)
        self.t_counts = torch.zeros(N, dtype=torch.int32, device=dev)
        self.t_status = torch.tensor([STATUS_CODES[self.trust.get_node_status(i)] for i in range(N)],
                                     dtype=torch.int32, device=dev)
        self.t_weights = torch.tensor(self.trust.weights_vector(), dtype=torch.float32, device=dev)
        self.t_recovery = torch.full((N,), self.trust.recovery_rate, dtype=torch.float32, device=dev)
        self.t_flagrun = torch.zeros(N, dtype=torch.int32, device=dev)
        # per replica: steps left in the grace window after a pipeline-wide anomaly
        self.t_grace = torch.zeros(max(1, self.dp), dtype=torch.float32, device=dev)
        # per node: weights failed the integrity check and have not been restored since (their
        # downstream output anomalies are echoes of that, not new Byzantine stages)
        self.t_taint = torch.zeros(N, dtype=torch.float32, device=dev)

    # ================================================================== helpers
    def my_stage(self) -> Optional[Stage]:
        if self.distributed:
            return self.stages.get(self.rank)
        return None

    def _stage_input(self, x: torch.Tensor, st: Stage) -> torch.Tensor:
        x = x.to(st.device, non_blocking=True)
        return x.to(self.dtype) if x.is_floating_point() else x

    def _host_metric_row(self, node: int) -> List[float]:
        return self._host_metrics.get(node, [0.0, 0.0, 0.0, 1.0])

    # ================================================================== training step
    REPORT_LAG = 2

    def train_step(self, batch: Dict[str, torch.Tensor]) -> Optional[float]:
        """One optimizer step over the global batch.  Returns the most recent loss the host has
        read: step reports are consumed exactly ``REPORT_LAG`` steps later on every rank (so the
        host never stalls the device queue, and collective decisions such as a re-shard happen
        at the same step everywhere); ``flush()`` drains the rest.

        ``TDL_COMPUTE_PRIORITY=high`` (A/B): the step's compute runs on a high-priority HIP stream,
        so the verification side stream's kernels take CUs only where the compute leaves them."""
        hi = self._priority_stream()
        if hi is None:
            return self._train_step(batch)
        cur = torch.cuda.current_stream(self.device)
        hi.wait_stream(cur)
        with torch.cuda.stream(hi):
            out = self._train_step(batch)
        cur.wait_stream(hi)
        return out

    def _priority_stream(self):
        if self.device.type != "cuda" or os.environ.get("TDL_COMPUTE_PRIORITY", "") != "high":
            return None
        s = getattr(self, "_hi_stream", None)
        if s is None:
            lo, hi = torch.cuda.Stream.priority_range()
            s = self._hi_stream = torch.cuda.Stream(self.device, priority=hi)
        return s

    def _train_step(self, batch: Dict[str, torch.Tensor]) -> Optional[float]:
        self.begin_step()
        progress.mark(f"step {self.global_step}: pipeline schedule")
        t0 = time.perf_counter()
        truth: Dict[int, bool] = {}
        self._truth_now = truth
        if self.attacker is not None and hasattr(self.attacker, "apply_attacks"):
            batch = self.attacker.apply_attacks(batch, self.global_step)
            truth.update(getattr(self.attacker, "last_batch_truth", {}) or {})
        M = self.cfg.micro_batches
        inp, tgt = batch["input"], batch["target"]
        if self.dp > 1:
            inp, tgt = inp.chunk(self.dp, 0)[self.replica], tgt.chunk(self.dp, 0)[self.replica]
        inputs = split_micro(inp, M)
        targets = split_micro(tgt, M)
        oc = self.cfg.output_check
        self._mon_idx = -1 if oc == "none" else (self._mon_rng.randrange(M) if oc == "random" else 0)
        # audited steps: WHETHER a step is audited and WHICH micro-batch are the auditor's private
        # choice (local: the engine's private RNG; distributed: each auditor's own RNG, revealed to
        # the auditee through the c10d store only after its outputs were sent — a step-hash
        # decision, as in round 3, was predictable by the auditee: ADVICE r3)
        self._audit_now = bool(self.cfg.audit and self.plan.num_stages > 1)
        if self._audit_now and not self.distributed and (
                self._mon_idx < 0 or (self.cfg.audit_prob < 1.0 and self._mon_rng.random() >= self.cfg.audit_prob)):
            self._audit_now = False
        tg = self.cfg.audit_targeted
        self._targeted = self._audit_now and M > 1 and (not self.distributed if tg is None else bool(tg))
        self._audit_rec: Dict[int, Dict[str, Any]] = {}
        self._audit_inputs: Dict[int, torch.Tensor] = {}   # distributed: this stage's received inputs
        self._audit_sent_dx: Dict[int, torch.Tensor] = {}  # distributed: input gradients sent upstream
        self._audit_recv_dy: Dict[int, torch.Tensor] = {}  # distributed: output gradients received
        self._audit_batch = inputs
        self._audit_targets = targets
        self._begin_commitments(len(inputs))
        if self.distributed:
            loss = self._run_1f1b(inputs, targets, truth)
        else:
            loss = self._run_local(inputs, targets, truth)
        self._finish_step(loss, truth)
        self.tracer.end_step(self.global_step)
        self.tracer.resolve()
        self._step_time = time.perf_counter() - t0
        return self.last_loss

    # ------------------------------------------------------------------ gradient commitments
    def _sketch_for(self, st: Stage):
        """The stage's gradient sketch (security/grad_audit.py), identical for the stage and any
        mirror of it (same layer range -> same flat layout, signs and tied-weight mask)."""
        from ..security.grad_audit import GradSketch, tied_ranges
        key = (tuple(st.layer_range), st.flat.numel, str(st.device))
        cache = self.__dict__.setdefault("_gsk_cache", {})
        sk = cache.get(key)
        if sk is None:
            tied = []
            for grp in self.ties:
                for li, attr in grp:
                    prm = st.local_param(li, attr)
                    if prm is not None:
                        tied.append(id(prm))
            a, b = st.layer_range
            sk = cache[key] = GradSketch(st.flat.numel, st.device, seed=self.cfg.seed * 1_000_003 + a * 7919 + b,
                                         masked=tied_ranges(st.flat, tied))
        return sk

    def _tied_param(self, st: Stage) -> Optional[torch.Tensor]:
        """This stage's member of the first tie group (GPT-2: wte / LM head), if any."""
        if not self.ties:
            return None
        for li, attr in self.ties[0]:
            prm = st.local_param(li, attr)
            if prm is not None:
                return prm
        return None

    def _tied_sketch(self, st: Stage, g: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
        """Sketch of the tied weight's gradient with a pattern shared by every member of the tie
        group (parameter-local indexing), so the members' sketches add up across stages."""
        from ..security.grad_audit import GradSketch
        prm = self._tied_param(st)
        if prm is None or getattr(prm, "main_grad", None) is None:
            return None
        cache = self.__dict__.setdefault("_tsk_cache", {})
        key = (prm.numel(), str(st.device))
        sk = cache.get(key)
        if sk is None:
            sk = cache[key] = GradSketch(prm.numel(), st.device, seed=self.cfg.seed * 7 + 424242)
        return sk((prm.main_grad if g is None else g).reshape(-1), sk.offset(self.cfg.seed, self.global_step))

    def _note_tied_pre(self, st: Stage):
        """Right before the tied all-reduce: the stage's own tied-weight gradient contribution."""
        if getattr(self, "_gsk_on", False):
            t = self._tied_sketch(st)
            if t is not None:
                self._tsk_pre[st.stage_id] = t

    def _begin_commitments(self, M: int):
        """Per-step running gradient sketches of every local stage (index 0: before the first
        micro-batch's backward, i + 1: after micro-batch i's weight gradients are accumulated)."""
        self._gsk_on = bool(self.cfg.audit and self.cfg.audit_backward and self.plan.num_stages > 1 and self.dp == 1)
        self._gsk_run: Dict[int, torch.Tensor] = {}
        self._tsk_pre: Dict[int, torch.Tensor] = {}
        if not self._gsk_on:
            return
        for node, st in self.stages.items():
            sk = self._sketch_for(st)
            r = torch.zeros(M + 1, 2, dtype=torch.float32, device=st.device)
            r[0].copy_(sk(st.flat.grad, sk.offset(self.cfg.seed, self.global_step)))
            self._gsk_run[node] = r

    def _commit_micro(self, node: int, st: Stage, i: int):
        """Micro-batch ``i``'s weight gradients of ``node`` are accumulated: (attack hook, then)
        commit the running sketch."""
        M = len(self._audit_batch)
        if self.attacker is not None and hasattr(self.attacker, "after_micro_backward"):
            if self.attacker.after_micro_backward(node, st.flat.grad, self.global_step, i, M):
                self._truth_now[node] = True
        r = self._gsk_run.get(node)
        if r is not None:
            sk = self._sketch_for(st)
            r[i + 1].copy_(sk(st.flat.grad, sk.offset(self.cfg.seed, self.global_step)))

    def _pre_micro(self, node: int, st: Stage, i: int):
        if self.attacker is not None and hasattr(self.attacker, "before_micro_backward"):
            self.attacker.before_micro_backward(node, st.flat.grad, self.global_step, i, len(self._audit_batch))

    def _tamper_dx(self, node: int, dx: torch.Tensor, i: int) -> torch.Tensor:
        """The input gradient ``node`` sends upstream for micro-batch ``i`` (Byzantine backward hook)."""
        if self.attacker is not None and hasattr(self.attacker, "on_input_grad"):
            d2 = self.attacker.on_input_grad(node, dx, self.global_step, i, len(self._audit_batch))
            if d2 is not None:
                self._truth_now[node] = True
                return d2
        return dx

    def begin_step(self) -> int:
        """Open an optimizer step (``train_step`` does this itself; the reference per-phase API —
        DistributedTrainer.forward_pass / backward_pass / optimizer_step — calls it explicitly)."""
        self._consume_reports(upto=self.global_step + 1 - self.REPORT_LAG)
        bump_weight_generation()   # weights may have changed since the last step (update, re-shard, restore, load)
        self._gsk_on = False       # the per-phase API (external backward) commits no gradient sketches
        self._truth_now = {}
        self.global_step += 1
        self.trust.advance_step(self.global_step)
        return self.global_step

    def end_step(self, loss: Optional[torch.Tensor], truth: Optional[Dict[int, bool]] = None) -> Optional[float]:
        """Close a step whose gradients are already accumulated in the stages' flat buffers (by an
        external ``loss.backward()``): tied all-reduce, verification digest, attribution, trust
        update, global-norm clipping + quarantine, fused AdamW — the same tail as ``train_step``."""
        self._finish_step(None if loss is None else loss.detach(), dict(truth or {}))
        self.tracer.end_step(self.global_step)
        self.tracer.resolve()
        return self.last_loss

    # ------------------------------------------------------------------ attacks on a stage
    def _attack_params(self, node: int, st: Stage, truth: Dict[int, bool]):
        if self.attacker is not None and hasattr(self.attacker, "on_parameters"):
            if self.attacker.on_parameters(node, st.flat, self.global_step):
                truth[node] = True
        # the stage's weights are final for this step from here on: take the integrity checksum now,
        # on the verifier's side stream, overlapped with the forward / backward instead of serially
        # on the step's tail (_integrity_flag picks it up after finish_step joined the side stream)
        side = getattr(st.verifier, "side", None)
        if self.cfg.param_integrity and side is not None and st.flat.data.is_cuda:
            cur = torch.cuda.current_stream(st.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                st._early_checksum = dstats.checksum(st.flat.data)
            st._early_checksum.record_stream(cur)

    def _attack_output(self, node: int, y: torch.Tensor, truth: Dict[int, bool], micro: Optional[int] = None,
                       num_micro: Optional[int] = None) -> torch.Tensor:
        if self.attacker is not None and hasattr(self.attacker, "on_output"):
            y2 = self.attacker.on_output(node, y, self.global_step, micro, num_micro)
            if y2 is not None:
                truth[node] = True
                return y2
        return y

    def _attack_grads(self, node: int, st: Stage, truth: Dict[int, bool]):
        if self.attacker is not None and hasattr(self.attacker, "on_gradients"):
            if self.attacker.on_gradients(node, st.flat.grad, self.global_step):
                truth[node] = True

    # ------------------------------------------------------------------ local (in-process) schedule
    def _run_local(self, inputs, targets, truth) -> Optional[torch.Tensor]:
        order = list(zip(self.plan.ranks, self.plan.ranges))
        M = len(inputs)
        for node, _ in order:
            self._attack_params(node, self.stages[node], truth)
        total = None
        bwd_audit = self._audit_now and self.cfg.audit_backward
        for i in range(M):
            x = inputs[i]
            watch = i == self._mon_idx
            for sidx, (node, _) in enumerate(order):
                st = self.stages[node]
                x = self._stage_input(x, st) if sidx == 0 else x.to(st.device, non_blocking=True)
                labels = targets[i].to(st.device, non_blocking=True) if st.computes_loss else None
                obs = st.output_observer() if watch else None
                rec = self._audit_rec.setdefault(node, {}).setdefault(i, {}) \
                    if self._audit_now and (watch or self._targeted) else None
                if rec is not None:
                    rec["x"] = x.detach().clone()
                    if st.computes_loss:
                        rec["labels"] = labels
                if sidx > 0 and x.requires_grad:
                    # the input gradient this stage sends upstream (Byzantine-backward hook first, then
                    # the audit's copy of what was sent); registered before the previous stage's
                    # output-gradient capture below, so that capture sees the gradient as sent
                    def _dx_hook(g, node=node, i=i, rec=rec):
                        g2 = self._tamper_dx(node, g, i)
                        if rec is not None and bwd_audit:
                            rec["dx"] = g2.detach().clone()
                        return g2 if g2 is not g else None
                    x.register_hook(_dx_hook)
                    prec = self._audit_rec.get(order[sidx - 1][0], {}).get(i) if rec is not None and bwd_audit else None
                    if prec is not None:
                        def _dy_hook(g, prec=prec):
                            prec["dy"] = g.detach().clone()
                        x.register_hook(_dy_hook)
                with self.tracer.phase("fwd"):
                    y, mon = st.forward(x, labels, observe=obs, arm_grad_stats=i == M - 1)
                if not st.computes_loss:
                    y = self._attack_output(node, y, truth, i, M)
                    if watch:
                        mon = y
                    if rec is not None:
                        rec["y"] = y.detach().clone()
                        if self._targeted:
                            rec["ystat"] = self._output_stat(rec["y"])
                if watch and mon is not None:
                    st.verifier.observe_output(mon)
                    if st.computes_loss and st.verifier.side is not None:
                        torch.cuda.current_stream(st.device).wait_stream(st.verifier.side)
                x = y
            loss = x / M
            for node, _ in order:
                self._pre_micro(node, self.stages[node], i)
            with self.tracer.phase("bwd_input"):
                loss.backward()
            for node, _ in order:
                self._commit_micro(node, self.stages[node], i)
            total = loss.detach() if total is None else total + loss.detach()
        return total

    # ------------------------------------------------------------------ distributed 1F1B schedule
    def _run_1f1b(self, inputs, targets, truth) -> Optional[torch.Tensor]:
        if self.p2p_mode == "async":
            return self._run_1f1b_async(inputs, targets, truth)
        st = self.my_stage()
        if st is None:
            return None
        node = self.rank
        comm = self.comm
        M = len(inputs)
        S = self.plan.num_stages
        s = st.stage_id
        first, last = s == 0, s == S - 1
        self._attack_params(node, st, truth)
        self._audit_early_ship(st)
        in_shape, out_shape = self._boundary_shapes(st, inputs[0])
        act_dtype = self.dtype
        defer_w = self.cfg.defer_wgrad and not first
        warm = min(S - s - 1, M)
        rem = M - warm
        in_q: deque = deque()
        out_q: deque = deque()
        total = [None]
        waited0 = comm.wait_seconds
        keep_out = self._audit_now and self.cfg.audit_backward and s == S - 2
        self._audit_outputs: Dict[int, torch.Tensor] = {}

        def get_input(i):
            if first:
                return self._stage_input(inputs[i], st)
            progress.mark(f"step {self.global_step}: stage {s} grouped exchange with rank {comm.prev}")
            x, _ = comm.exchange(recv_prev=(in_shape, act_dtype))
            return x

        def fwd(i, x):
            if not first:
                x.requires_grad_(True)
            labels = targets[i].to(st.device, non_blocking=True) if last else None
            watch = i == self._mon_idx
            obs = st.output_observer() if watch else None
            if self._audit_now and not first:
                # every received input stays referenced until the audit (no copy): it is the previous
                # stage's output as seen here (audited here) and my input (the next stage audits me)
                self._audit_inputs[i] = x.detach()
            y, mon = st.forward(x, labels, observe=obs, arm_grad_stats=i == M - 1 and not defer_w)
            if last:
                y = y / M
                total[0] = y.detach() if total[0] is None else total[0] + y.detach()
            else:
                y = self._attack_output(node, y, truth, i, M)
                if watch:
                    mon = y
                if keep_out:
                    self._audit_outputs[i] = y.detach()
            if watch and mon is not None:
                st.verifier.observe_output(mon)
                if last and st.verifier.side is not None:
                    # the CE backward rewrites the logits buffer in place
                    torch.cuda.current_stream(st.device).wait_stream(st.verifier.side)
            return y

        def bwd(bi, x, y, dy):
            """Input-gradient backward; the weight-gradient GEMMs are queued (ops.layers
            .defer_weight_grads) and run by the caller AFTER dx has been posted upstream."""
            self._pre_micro(node, st, bi)
            if dy is not None and self._audit_now:
                self._audit_recv_dy[bi] = dy
            with defer_weight_grads(defer_w) as dw:
                if last:
                    y.backward()
                else:
                    torch.autograd.backward(y, dy)
            dx = None
            if not first:
                dx = self._tamper_dx(node, x.grad, bi)
                if self._audit_now:
                    self._audit_sent_dx[bi] = dx
            dw.bi = bi
            return dx, dw

        def wgrad(dw):
            dw.run()
            self._commit_micro(node, st, dw.bi)

        def send_dx_then_w(dx, dw, recv_prev=None):
            h = comm.post(send_prev=dx, recv_prev=recv_prev)
            wgrad(dw)  # overlaps the transfer and the upstream stage's backward
            return comm.wait(h)[0]

        for i in range(warm):
            x = get_input(i)
            y = fwd(i, x)
            comm.exchange(send_next=y)
            in_q.append((i, x))
            out_q.append(y)
        x = get_input(warm) if rem > 0 else None
        for j in range(rem):
            i = warm + j
            y = fwd(i, x)
            if last:
                dy = None
            else:
                _, dy = comm.exchange(send_next=y, recv_next=(out_shape, act_dtype))
            in_q.append((i, x))
            out_q.append(y)
            (bi, x0), y0 = in_q.popleft(), out_q.popleft()
            dx, dw = bwd(bi, x0, y0, dy)
            if j == rem - 1:
                if not first:
                    send_dx_then_w(dx, dw)
                else:
                    wgrad(dw)
            else:
                if first:
                    wgrad(dw)
                    x = get_input(i + 1)
                else:
                    x = send_dx_then_w(dx, dw, recv_prev=(in_shape, act_dtype))
        for _ in range(warm):
            (bi, x0), y0 = in_q.popleft(), out_q.popleft()
            dy = None
            if not last:
                _, dy = comm.exchange(recv_next=(out_shape, act_dtype))
            dx, dw = bwd(bi, x0, y0, dy)
            if not first:
                send_dx_then_w(dx, dw)
            else:
                wgrad(dw)
        self._comm_wait = comm.wait_seconds - waited0
        return total[0]

    def _run_1f1b_async(self, inputs, targets, truth) -> Optional[torch.Tensor]:
        """1F1B with latency-hiding point-to-point transfers.

        Activations travel on one process group and activation gradients on another, so every
        communicator carries one-way traffic per neighbour pair in issue order (deadlock-free for
        any interleaving of the two directions).  Each receive is posted one compute phase ahead
        of its use — the next input before this stage's backward, the next output gradient before
        its forward — so the xGMI transfer overlaps compute instead of adding a full transfer
        latency to every pipeline hop (the grouped exchange serialises send and receive behind
        both neighbours' compute).  On each direction's stream a send is always issued before the
        next receive, so a ready send never queues behind a pending receive.  The compute stream
        never waits for a send; all sends are drained at the end of the step.  Weight gradients
        (B/W split) run after the input gradient is posted."""
        st = self.my_stage()
        if st is None:
            return None
        node = self.rank
        M = len(inputs)
        S = self.plan.num_stages
        s = st.stage_id
        first, last = s == 0, s == S - 1
        self._attack_params(node, st, truth)
        self._audit_early_ship(st)
        in_shape, out_shape = self._boundary_shapes(st, inputs[0])
        act_pg, grad_pg = self._dir_groups
        prev, nxt = self.comm.prev, self.comm.next
        dt = self.dtype
        warm = min(S - s - 1, M)
        rem = M - warm
        in_q: deque = deque()
        out_q: deque = deque()
        sends: List = []
        total = [None]
        waited = [0.0]
        defer_w = self.cfg.defer_wgrad and not first
        # the stage before the loss stage audits it and needs its own outputs (the loss stage's inputs)
        keep_out = self._audit_now and self.cfg.audit_backward and s == S - 2
        self._audit_outputs: Dict[int, torch.Tensor] = {}

        step = self.global_step

        def post_recv(shape, src, group):
            buf = torch.empty(shape, dtype=dt, device=st.device)
            return p2p.irecv(buf, src, group=group), buf, src

        def take(h):
            progress.mark(f"step {step}: stage {s} waits for a P2P receive from rank {h[2]}")
            t0 = time.perf_counter()
            h[0].wait()
            waited[0] += time.perf_counter() - t0
            progress.mark(f"step {step}: stage {s} compute")
            return h[1]

        def post_x(i):
            return None if first or i >= M else post_recv(in_shape, prev, act_pg)

        def post_dy(i):
            return None if last or i >= M else post_recv(out_shape, nxt, grad_pg)

        def send(t, dst, group):
            sends.append(p2p.isend(t.contiguous(), dst, group=group))
            if len(sends) > 8:  # drop finished sends (their tensors are released)
                sends[:] = [w for w in sends if not w.is_completed()]

        def fwd(i, x):
            if not first:
                x.requires_grad_(True)
            labels = targets[i].to(st.device, non_blocking=True) if last else None
            watch = i == self._mon_idx
            obs = st.output_observer() if watch else None
            if self._audit_now and not first:
                # every received input stays referenced until the audit (no copy): it is the previous
                # stage's output as seen here (audited here) and my input (the next stage audits me)
                self._audit_inputs[i] = x.detach()
            y, mon = st.forward(x, labels, observe=obs, arm_grad_stats=i == M - 1 and not defer_w)
            if last:
                y = y / M
                total[0] = y.detach() if total[0] is None else total[0] + y.detach()
            else:
                y = self._attack_output(node, y, truth, i, M)
                if watch:
                    mon = y
                if keep_out:
                    self._audit_outputs[i] = y.detach()
            if watch and mon is not None:
                st.verifier.observe_output(mon)
                if last and st.verifier.side is not None:
                    torch.cuda.current_stream(st.device).wait_stream(st.verifier.side)
            return y

        def bwd(bi, x, y, dy):
            self._pre_micro(node, st, bi)
            if dy is not None and self._audit_now:
                self._audit_recv_dy[bi] = dy
            with defer_weight_grads(defer_w) as dw:
                if last:
                    y.backward()
                else:
                    torch.autograd.backward(y, dy)
            dx = None
            if not first:
                dx = self._tamper_dx(node, x.grad, bi)
                if self._audit_now:
                    self._audit_sent_dx[bi] = dx
            return dx, dw

        def wgrad(bi, dw):
            dw.run()
            self._commit_micro(node, st, bi)

        def input_of(i, h):
            return self._stage_input(inputs[i], st) if first else take(h)

        tr = self.tracer
        if tr.enabled:
            fwd, bwd, take = tr.wrap("fwd", fwd), tr.wrap("bwd_input", bwd), tr.wrap("p2p_wait", take)

        x_h = post_x(0)
        for i in range(warm):                      # warm > 0 implies not last
            x = input_of(i, x_h)
            y = fwd(i, x)
            send(y, nxt, act_pg)
            x_h = post_x(i + 1)
            in_q.append((i, x))
            out_q.append(y)
        for j in range(rem):
            i = warm + j
            x = input_of(i, x_h)
            dy_h = post_dy(j)                      # arrives while this forward runs
            y = fwd(i, x)
            if not last:
                send(y, nxt, act_pg)
            x_h = post_x(i + 1)                    # arrives while the backward below runs
            in_q.append((i, x))
            out_q.append(y)
            (bi, x0), y0 = in_q.popleft(), out_q.popleft()
            dy = None if last else take(dy_h)
            dx, dw = bwd(bi, x0, y0, dy)
            if not first:
                send(dx, prev, grad_pg)
            with tr.phase("bwd_weight"):
                wgrad(bi, dw)
        dy_h = post_dy(rem) if warm > 0 else None
        for c in range(warm):
            b = rem + c
            dy = take(dy_h)
            (bi, x0), y0 = in_q.popleft(), out_q.popleft()
            dx, dw = bwd(bi, x0, y0, dy)
            if not first:
                send(dx, prev, grad_pg)
            dy_h = post_dy(b + 1)                  # after the send: no send queues behind it
            with tr.phase("bwd_weight"):
                wgrad(bi, dw)
        progress.mark(f"step {step}: stage {s} drains its P2P sends")
        t0 = time.perf_counter()
        for w in sends:
            w.wait()
        waited[0] += time.perf_counter() - t0
        self._comm_wait = waited[0]
        return total[0]

    def _boundary_shapes(self, st: Stage, sample_in: torch.Tensor):
        """Activation shapes entering / leaving this stage (exchanged once, then cached)."""
        key = (self.plan.version, tuple(sample_in.shape))
        cached = getattr(self, "_shape_cache", {}).get(key)
        if cached is not None:
            return cached
        S = self.plan.num_stages
        s = st.stage_id
        hdr = torch.zeros(8, dtype=torch.int64, device=st.device)
        in_shape = None
        if s > 0:
            h, _ = self.comm.exchange(recv_prev=((8,), torch.int64))
            note_host_sync()
            in_shape = torch.Size([int(v) for v in h[1:1 + int(h[0])].tolist()])
            probe = torch.zeros(in_shape, dtype=self.dtype, device=st.device)
        else:
            probe = sample_in.to(st.device)
        out_shape = None
        if s < S - 1:
            was_training = st.module.training
            st.module.eval()  # shape probe must not touch BatchNorm running statistics
            with torch.no_grad():
                y, _ = st.forward(probe, None)
            st.module.train(was_training)
            out_shape = y.shape
            hdr[0] = len(out_shape)
            hdr[1:1 + len(out_shape)] = torch.tensor(list(out_shape), dtype=torch.int64)
            self.comm.exchange(send_next=hdr)
        if not hasattr(self, "_shape_cache"):
            self._shape_cache = {}
        self._shape_cache[key] = (in_shape, out_shape)
        return in_shape, out_shape

    # ------------------------------------------------------------------ step epilogue
    def _tied_grad(self):
        st = self.my_stage()
        if st is None:
            return None
        for grp in self.ties:
            for li, attr in grp:
                p = st.local_param(li, attr)
                if p is not None:
                    return p.main_grad
        return None

    def _launch_tied_allreduce(self):
        """Called from the autograd hook that sees this stage's tied weight's last gradient
        contribution of the step (the LM head's, early in the last stage's final backward): the
        tied-gradient all-reduce starts right away on its communicator's stream, overlapping the
        rest of the backward, instead of after the drain.  The embedding's side joins when its
        gradient is final (its backward is the stage's last); ``_allreduce_tied`` waits."""
        if getattr(self, "_tie_work", None) is not None or not self.tie_members or self.rank not in self.tie_members:
            return
        g = self._tied_grad()
        if g is not None:
            st = self.my_stage()
            if st is not None:
                self._note_tied_pre(st)
            if g.is_cuda:   # a weight gradient still running on the side stream (ops/side_stream.py)
                from ..ops.side_stream import wait_wgrad
                wait_wgrad(torch.cuda.current_stream(g.device), g.device)
            self._tie_work = dist.all_reduce(g, group=self.tie_group, async_op=True)

    def _allreduce_tied(self):
        if not self.ties:
            return
        work = getattr(self, "_tie_work", None)
        if work is not None:
            self._tie_work = None
            work.wait()
            return
        if not self.distributed:
            # local mode: tied copies on different stages -> sum their grads into both
            for grp in self.ties:
                owners = [(self.plan.owner_of_layer(li), li, attr) for li, attr in grp]
                params = []
                for node, li, attr in owners:
                    p = self.stages[node].local_param(li, attr)
                    if all(p is not q for q in params):
                        params.append(p)
                if len(params) > 1:
                    for node, _, _ in owners:
                        self._note_tied_pre(self.stages[node])
                    tot = sum(p.main_grad.to(params[0].device) for p in params)
                    for p in params:
                        p.main_grad.copy_(tot.to(p.device))
            return
        if not self.tie_members or self.rank not in self.tie_members:
            return
        st = self.my_stage()
        # one all-reduce per tie group, in the same order on every member (the early path handles
        # only the first group: it is used only when there is exactly one)
        for gi, grp in enumerate(self.ties):
            for li, attr in grp:
                p = st.local_param(li, attr)
                if p is not None:
                    if gi == 0:
                        self._note_tied_pre(st)
                    dist.all_reduce(p.main_grad, group=self.tie_group)
                    break

    def _index_tensor(self, nodes) -> torch.Tensor:
        """Device index tensor of a node list, cached per list (building it is a blocking pageable
        host-to-device copy; the present set only changes on a re-plan or an OFFLINE event)."""
        key = tuple(nodes)
        cache = self.__dict__.setdefault("_idx_cache", {})
        t = cache.get(key)
        if t is None:
            t = cache[key] = torch.tensor(list(key), dtype=torch.long, device=self.device)
        return t

    def _finish_step(self, loss, truth: Dict[int, bool]):
        tv = self.tracer.begin("verify")
        progress.mark(f"step {self.global_step}: tied-weight gradient all-reduce")
        self._allreduce_tied()
        N = self.num_nodes
        rows = []
        for node, st in self.stages.items():
            self._attack_grads(node, st, truth)
            hm = self._host_metric_row(node)
            d = st.verifier.finish_step(st.flat.grad, loss if st.computes_loss else None, hm,
                                        truth.get(node, False), st.stage_id)
            # the weight commitment made after this stage's last update (before anything of this
            # step could touch the weights): the auditor checks the weights it receives against it
            pc = getattr(st, "param_checksum", None)
            if pc is not None and self.cfg.audit and self.plan.num_stages > 1:
                from ..security.grad_audit import fold_hash
                d[SV.D_WHASH:SV.D_WHASH + 2].copy_(fold_hash(pc))
            else:
                d[SV.D_WHASH:SV.D_WHASH + 2].fill_(-1.0)
            if self.cfg.param_integrity:
                d[SV.D_PARAM_FLAG:SV.D_PARAM_FLAG + 1].copy_(self._integrity_flag(st))
                if self.attacker is not None and getattr(self.attacker, "lies_about_integrity", None) \
                        and self.attacker.lies_about_integrity(node, self.global_step):
                    d[SV.D_PARAM_FLAG:SV.D_PARAM_FLAG + 1].fill_(0.0)   # a rank lying about its own check
            self._write_commitments(node, st, d)
            rows.append((node, d))
        if getattr(self, "_audit_now", False):
            ta = self.tracer.begin("audit")
            progress.mark(f"step {self.global_step}: recompute audit")
            t_a = time.perf_counter()
            ev = None
            if self.device.type == "cuda":
                ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                ev[0].record()
            self._audit(dict(rows))
            if ev is not None:
                ev[1].record()
            self._note_audit_cost(time.perf_counter() - t_a, ev)
            self.tracer.end(ta)
        if self.distributed:
            mine = rows[0][1] if rows else torch.zeros(SV.DIGEST, dtype=torch.float32, device=self.device)
            if self.heartbeat is not None:
                mine[SV.D_OFFLINE_MASK:SV.D_OFFLINE_MASK + 1].fill_(
                    float(sum(1 << n for n in self.heartbeat.offline() if n < 24)))
            progress.mark(f"step {self.global_step}: digest all-gather")
            D = all_gather_rows(mine, self.world)
            if self.heartbeat is not None:
                self._apply_offline(D)
        else:
            D = torch.zeros(N, SV.DIGEST, dtype=torch.float32, device=self.device)
            for node, d in rows:
                D[node].copy_(d.to(self.device))
        blame, evidence = self._attribute(D)
        if self.quarantine_on_evidence:
            # a tampered forward (output anomaly / failed integrity check anywhere in the pipeline)
            # taints every gradient of the step: skip the update on all of the replica's stages, so
            # the damage does not echo into the next step's outputs
            for node, st in self.stages.items():
                st.verifier.ctrl[1:2].copy_(torch.maximum(st.verifier.ctrl[1:2], evidence[node:node + 1].to(st.device)))
        if self.dp > 1:
            total_sumsq = self._dp_aggregate(D, evidence)
        else:
            # global gradient norm for clipping: sum of the per-stage sumsq of the updates that will
            # be applied (each tied weight counted once, quarantined stages left out); every rank
            # computes it from the same all-gathered digest
            sq = D[:, SV.D_GRAD_SUMSQ]
            if self.quarantine_on_evidence:
                sq = sq * (1.0 - evidence)
            total_sumsq = sq.sum()
        present_nodes = self.all_ranks()
        idx = self._index_tensor(present_nodes)
        raw = blame.to(torch.int32)
        # a single flag quarantines that step's update; k consecutive flags compromise the node;
        # a failed weight-integrity check (weights rewritten outside the optimizer) is definitive
        # evidence and compromises at once
        self.t_flagrun.copy_((self.t_flagrun + 1) * raw)
        proof = self._proof if self.cfg.compromise_on_proof else (D[:, SV.D_PARAM_FLAG] > 0).float()
        flags = torch.maximum((self.t_flagrun >= max(1, self.cfg.compromise_after)).to(torch.int32),
                              (proof > 0).to(torch.int32) * raw)
        # every blamed step also costs trust through the metrics (worst output deviation, no
        # gradient consistency), so isolated detections accumulate instead of being forgotten
        metrics = D[:, SV.D_METRICS:SV.D_METRICS + 6].clone()
        metrics[:, 0] = torch.maximum(metrics[:, 0], blame)
        metrics[:, 1] = metrics[:, 1] * (1.0 - blame)
        if len(present_nodes) == N:
            dstats.trust_update(self.t_values, self.t_counts, self.t_status, metrics, self.t_weights,
                                self.trust.trust_threshold, self.cfg.trust_decay_per_step, 1.0,
                                flags.contiguous(), self.t_recovery)
        else:
            v, c, s_ = self.t_values[idx].clone(), self.t_counts[idx].clone(), self.t_status[idx].clone()
            dstats.trust_update(v, c, s_, metrics[idx].contiguous(), self.t_weights, self.trust.trust_threshold,
                                self.cfg.trust_decay_per_step, 1.0, flags[idx].contiguous(),
                                self.t_recovery[idx].contiguous())
            self.t_values[idx] = v
            self.t_counts[idx] = c
            self.t_status[idx] = s_
        self.tracer.end(tv)
        progress.mark(f"step {self.global_step}: optimizer")
        to = self.tracer.begin("optimizer")
        for node, st in self.stages.items():
            st.verifier.set_clip_scale(total_sumsq.to(st.device), self.cfg.adamw.max_grad_norm)
            cur = getattr(st, "_cur_checksum", None)
            if self.cfg.param_integrity and cur is not None:
                # the weights must still be those checksummed at the start of the step
                st._tail_flag = (dstats.checksum(st.flat.data) != cur).any().float().reshape(1)
            st.flat.adamw_step(self.cfg.adamw, ctrl=st.verifier.ctrl)
            if self.cfg.param_integrity:
                st.param_checksum = dstats.checksum(st.flat.data, getattr(st, "param_checksum", None))
        self.tracer.end(to)
        if self._shadow_enabled() and self.global_step % self.cfg.shadow_interval == 0:
            self._take_shadow()
        if self.dp > 1 and self.cfg.param_audit_interval and self.global_step % self.cfg.param_audit_interval == 0:
            self._audit_params()
        # queue the host report (pinned, non-blocking)
        if getattr(self, "_audit_now", False):
            _, adone = self._audit_vectors(D)
        else:
            adone = torch.zeros(N, dtype=torch.float32, device=self.device)
        akind = self._proof_kind
        rep = torch.cat([D.reshape(-1), self.t_values, self.t_status.float(), blame.float(), akind, adone])
        if rep.is_cuda:
            host = torch.empty(rep.shape, dtype=rep.dtype, pin_memory=True)
            host.copy_(rep, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host, ev = rep.clone(), None
        self._pending.append((self.global_step, self.epoch, host, ev, dict(truth), list(self.last_ranks())))

    def _write_commitments(self, node: int, st: Stage, d: torch.Tensor):
        """Digest slots of the gradient commitments: the sketch of the gradient about to be applied
        (after the tied all-reduce and every hook) and the committed running sketch after the last
        micro-batch's backward.  They differ when the gradient was rewritten in between."""
        r = self._gsk_run.get(node) if getattr(self, "_gsk_on", False) else None
        if r is None:
            d[SV.D_GSK_ON:SV.D_GSK_ON + 1].fill_(0.0)
            return
        sk = self._sketch_for(st)
        d[SV.D_GSK_APP:SV.D_GSK_APP + 2].copy_(sk(st.flat.grad, sk.offset(self.cfg.seed, self.global_step)))
        d[SV.D_GSK_BWD:SV.D_GSK_BWD + 2].copy_(r[-1])
        d[SV.D_GSK_ON:SV.D_GSK_ON + 1].fill_(1.0)
        pre = self._tsk_pre.get(st.stage_id)
        if pre is not None:
            d[SV.D_TSK_PRE:SV.D_TSK_PRE + 2].copy_(pre)
            d[SV.D_TSK_APP:SV.D_TSK_APP + 2].copy_(self._tied_sketch(st))
            d[SV.D_TSK_ON:SV.D_TSK_ON + 1].fill_(1.0)
        else:
            d[SV.D_TSK_ON:SV.D_TSK_ON + 1].fill_(0.0)

    # ================================================================== deterministic stage cross-check
    def _recompute(self, st: Stage, x: torch.Tensor, dy: Optional[torch.Tensor] = None,
                   labels: Optional[torch.Tensor] = None, M: int = 1, backward: bool = False):
        """``st``'s forward of one micro-batch as in training (BatchNorm in batch-statistics mode),
        and with ``backward`` its backward from the output gradient ``dy`` (the loss stage: from
        its loss / M, as the schedule runs it), without leaving a trace: module buffers (running
        statistics) are restored and the weight gradients go to a scratch accumulator, whose
        sketch is returned.  Returns (output, input gradient or None, weight-gradient sketch or None)."""
        bufs = [b.detach().clone() for b in st.module.buffers()]
        try:
            if not backward:
                with torch.no_grad():   # no autograd graph / saved activations for the recompute
                    y, _ = st.forward(x, labels)
                return y, None, None
            scratch = torch.zeros_like(st.flat.grad)
            saved = st.flat.set_grad_buffer(scratch)
            try:
                xg = x.detach().clone()
                if xg.is_floating_point():
                    xg.requires_grad_(True)
                with torch.enable_grad():
                    y, _ = st.forward(xg, labels)
                    if st.computes_loss:
                        (y / M).backward()
                    else:
                        torch.autograd.backward(y, dy)
                sk = self._sketch_for(st)
                skv = sk(scratch, sk.offset(self.cfg.seed, self.global_step))
                dx = xg.grad if xg.is_floating_point() else None
                return y.detach(), dx, skv
            finally:
                st.flat.set_grad_buffer(saved)
        finally:
            with torch.no_grad():
                for b, v in zip(st.module.buffers(), bufs):
                    b.copy_(v)

    @staticmethod
    @torch.no_grad()
    def _output_stat(y: torch.Tensor):
        """(log RMS, token-mean vector over the last dim) of one micro-batch's stage output, device."""
        yf = y.float()
        return (yf.square().mean().clamp_min(1e-30).log().reshape(1),
                yf.reshape(-1, yf.shape[-1]).mean(0) if yf.dim() > 1 else yf.reshape(1, -1).mean(0))

    @torch.no_grad()
    def _target_scores(self, ystats, run) -> Optional[torch.Tensor]:
        """Robust |z| per micro-batch (max over the statistics) of: the output's log RMS, the cosine of
        its token-mean vector with the other micro-batches' (a sign flip or a large perturbation
        drives it toward -1 / 0) and the norm of its committed weight-gradient sketch contribution."""
        terms = []
        if ystats:
            lr = torch.cat([a for a, _ in ystats])
            V = torch.stack([v for _, v in ystats])
            ref = V.sum(0, keepdim=True) - V                      # the other micro-batches' sum
            cos = torch.nn.functional.cosine_similarity(V, ref, dim=1)
            terms += [(lr, 0.05), (cos, 0.05)]
        if run is not None and run.shape[0] > 2:
            dn = (run[1:] - run[:-1]).norm(dim=1).clamp_min(1e-30).log()
            terms.append((dn, 0.1))
        if not terms:
            return None
        zs = []
        for t, floor in terms:
            med = t.median()
            mad = (t - med).abs().median()
            zs.append((t - med).abs() / torch.clamp(1.4826 * mad, min=floor))
        return torch.stack(zs).amax(0)

    def _target_picks(self, order) -> Dict[int, int]:
        """Local mode: per audited stage, the micro-batch with the largest anomaly score if it
        exceeds ``audit_target_z`` (one device->host read for all stages)."""
        M = len(self._audit_batch)
        nodes, best = [], []
        for k, p in enumerate(order):
            recs = self._audit_rec.get(p, {})
            last = k == len(order) - 1
            ystats = None
            if not last:
                ystats = [recs.get(m, {}).get("ystat") for m in range(M)]
                if any(v is None for v in ystats):
                    ystats = None
            run = self._gsk_run.get(p) if getattr(self, "_gsk_on", False) else None
            z = self._target_scores(ystats, run)
            if z is None:
                continue
            nodes.append(p)
            best.append(torch.stack([z.max(), z.argmax().float()]).to(self.device))
        if not best:
            return {}
        vals = torch.stack(best).tolist()
        thr = self.cfg.audit_target_z
        picks = {p: int(i) for p, (zm, i) in zip(nodes, vals) if zm > thr}
        tl = self.__dict__.setdefault("_target_log", [])
        tl.extend((self.global_step, p, m) for p, m in picks.items())
        return picks

    def _audit_verdict(self, y_seen: torch.Tensor, y_ref: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(mismatch flag, relative max error) of a received output against its recomputation —
        device tensors, no host sync.  Non-finite values count as a mismatch."""
        a, b = y_seen.float(), y_ref.float()
        err = (a - b).abs().amax() / b.abs().amax().clamp_min(1e-12)
        err = torch.nan_to_num(err, nan=1e30, posinf=1e30)
        return (err > self.cfg.audit_tol).float().reshape(1), err.reshape(1)

    def _audit_one(self, st: Stage, x: torch.Tensor, m: int, M: int, y_seen=None, dy=None, labels=None,
                   dx_seen=None, run=None, whash=None):
        """All checks of one audited micro-batch ``m`` of stage ``st`` (its own modules in local mode,
        a mirror holding its shipped weights in distributed mode).  Returns device tensors
        (mismatch flag [1], failed-check bitmask [1], worst relative error [1]).

        * forward (AK_FWD): the output the next stage received == f(x; W);
        * input gradient (AK_DX): the gradient sent upstream == the recomputed one for the output
          gradient the audited stage received;
        * weight gradient (AK_DW): the sketch of micro-batch m's committed contribution
          (running sketches ``run[m+1] - run[m]``) == the sketch of the recomputed one;
        * weights (AK_WHASH, local mode): the weights in use == the stage's post-update commitment."""
        from ..security.grad_audit import sketch_mismatch
        bwd = self.cfg.audit_backward and (st.computes_loss or dy is not None)
        y_ref, dx_ref, sk_ref = self._recompute(st, x, dy, labels, M, backward=bwd)
        z = torch.zeros(1, dtype=torch.float32, device=st.device)
        kind, err = z.clone(), z.clone()
        if y_seen is not None and not st.computes_loss:
            f, e = self._audit_verdict(y_seen, y_ref)
            kind += f * SV.AK_FWD
            err = torch.maximum(err, e)
        if bwd and dx_seen is not None and dx_ref is not None:
            f, e = self._audit_verdict(dx_seen, dx_ref)
            kind += f * SV.AK_DX
            err = torch.maximum(err, e)
        if bwd and run is not None and sk_ref is not None and 0 <= m < run.shape[0] - 1:
            floor = 1e-3 * (run[1:] - run[:-1]).abs().amax()
            f, e = sketch_mismatch(run[m + 1] - run[m], sk_ref, self.cfg.audit_grad_tol, floor)
            kind += f * SV.AK_DW
            err = torch.maximum(err, e)
        if whash is not None:
            kind += whash * SV.AK_WHASH
        return (kind > 0).float(), kind, err

    def _audit(self, rows: Dict[int, torch.Tensor]):
        """Recompute audit of one privately chosen micro-batch per stage and step.

        Every non-loss stage is audited by the NEXT stage (it received the output and sent back the
        output gradient), the loss stage by its predecessor (which received its input gradient).
        Forward (the output equals f(input; weights)) and, with ``audit_backward``, backward (the
        input gradient sent upstream and the micro-batch's weight-gradient contribution equal their
        recomputation) — see ``_audit_one``.  Local mode: the engine holds every stage and computes
        each verdict right here.  Distributed: see ``_audit_dist``.  A verdict rides in its
        auditor's digest row (``D_AUDIT_PREV`` / ``D_AUDIT_NEXT``), so no collective is added; a
        tampered activation or gradient mismatches deterministically, a weight perturbation
        recomputes consistently but fails the weight commitment, a clean stage always matches."""
        if self.distributed:
            self._audit_dist(rows)
            return
        from ..security.grad_audit import fold_hash
        order = list(self.plan.ranks)
        S = len(order)
        M = len(self._audit_batch)
        picks = self._target_picks(order) if self._targeted else {}
        for k in range(S):
            p = order[k]
            last = k == S - 1
            if last and not self.cfg.audit_backward:
                continue
            aud = order[k + 1] if not last else order[k - 1]
            recs = self._audit_rec.get(p, {})
            chosen = [m for m in dict.fromkeys([self._mon_idx, picks.get(p, -1)]) if m >= 0 and "x" in recs.get(m, {})]
            if not chosen or aud not in rows:
                continue
            st = self.stages[p]
            wh = None
            cur, ref = getattr(st, "_cur_checksum", None), getattr(st, "param_checksum", None)
            if cur is not None and ref is not None and cur is not ref:
                wh = (fold_hash(cur) != fold_hash(ref)).any().float().reshape(1)
            flag = kind = err = None
            for m in chosen:
                rec = recs[m]
                f1, k1, e1 = self._audit_one(st, rec["x"], m, M, y_seen=rec.get("y"),
                                             dy=None if last else rec.get("dy"), labels=rec.get("labels"),
                                             dx_seen=rec.get("dx"), run=self._gsk_run.get(p), whash=wh)
                if flag is None:
                    flag, kind, err = f1, k1, e1
                else:   # failed-check bits of both audited micro-batches
                    flag, err = torch.maximum(flag, f1), torch.maximum(err, e1)
                    kind = torch.bitwise_or(kind.long(), k1.long()).float()
            d = rows[aud]
            base = (SV.D_AUDIT_NEXT, SV.D_AUDITED_NEXT, SV.D_AUDIT_KIND_NEXT) if last else \
                (SV.D_AUDIT_PREV, SV.D_AUDITED_PREV, SV.D_AUDIT_KIND_PREV)
            d[base[0]:base[0] + 1].copy_(flag.to(d.device))
            d[base[1]:base[1] + 1].fill_(1.0)
            d[base[2]:base[2] + 1].copy_(kind.to(d.device))
            d[SV.D_AUDIT_ERR:SV.D_AUDIT_ERR + 1].copy_(torch.maximum(d[SV.D_AUDIT_ERR:SV.D_AUDIT_ERR + 1],
                                                                    err.to(d.device)))

    def _audit_early_ship(self, st: Stage):
        """Distributed audit, weights part, posted BEFORE the 1F1B schedule on the audit
        communicator so the transfer overlaps the step instead of sitting in its tail (a stage of
        GPT-2-medium at 8 stages ships 75-180 MB of bf16 weights per step).  The weights sent are
        those of the step (posted after the attacker's parameter hook, nothing writes them before
        the optimizer, which runs after the audit waited for the transfer); shipping every step
        reveals nothing about the private choice, so this runs only when every step is audited
        (``audit_prob`` = 1).  ``_audit_dist`` waits for it and skips its own weight transfer."""
        self._early_ship = None
        if not (self.distributed and getattr(self, "_audit_now", False) and self.cfg.audit_prob >= 1.0
                and getattr(self, "_audit_pg", None) is not None):
            return
        s, S = st.stage_id, self.plan.num_stages
        prev, nxt = self.comm.prev, self.comm.next
        bwd = self.cfg.audit_backward
        my_auditor = nxt if nxt is not None else (prev if bwd and s == S - 1 and prev is not None else None)
        mirrors: Dict[str, Stage] = {}
        sends, recvs = [], []
        if my_auditor is not None:
            sends.append((st.flat.data, my_auditor))
        if prev is not None:
            mirrors["prev"] = self._audit_mirror(tuple(self.plan.ranges[s - 1]), s - 1)
            recvs.append((mirrors["prev"].flat.data, prev))
        if bwd and nxt is not None and s + 1 == S - 1:
            mirrors["next"] = self._audit_mirror(tuple(self.plan.ranges[s + 1]), s + 1)
            recvs.append((mirrors["next"].flat.data, nxt))
        if not sends and not recvs:
            return
        g = self._audit_pg
        ops = [dist.P2POp(dist.isend, t, r, g) for t, r in sends] + [dist.P2POp(dist.irecv, t, r, g) for t, r in recvs]
        a = self.__dict__.setdefault("_audit_cost", {"steps": 0, "host_s": 0.0, "bytes": 0, "events": []})
        a["bytes"] += sum(t.numel() * t.element_size() for t, _ in sends + recvs)
        self._early_ship = (dist.batch_isend_irecv(ops), mirrors)

    def _audit_dist(self, rows: Dict[int, torch.Tensor]):
        """Distributed audit protocol of one rank (stage s of S):

        1. commit: every audited stage sends its running gradient sketches (one [M+1, 2] tensor) to
           its auditor BEFORE any choice is revealed;
        2. reveal: each auditor draws privately whether to audit and which micro-batch (-1 = no
           audit) and posts it in the c10d store (host to host, no device sync); the auditee reads
           it only now, after every output and gradient of the step reached its peers;
        3. ship: the auditee sends its bf16 weights, and (non-first, non-loss stages) its input and
           the input gradient it sent upstream for that micro-batch; the loss stage ships only its
           weights (its auditor holds its input, the labels and the gradient it sent);
        4. verify on a mirror of the audited stage (``_audit_one``); the hash of the weights
           received (vs the auditee's post-update commitment ``D_WHASH``) and of the input gradient
           shipped (vs what the upstream stage received, ``D_DXHASH_RECV``) go into the auditor's
           row and are compared on every rank in ``_attribute`` — so a rank that lies about its own
           integrity check, or ships a different gradient than it sent, is still caught."""
        from ..security.grad_audit import hash2
        st = self.my_stage()
        if st is None:
            return
        s, S = st.stage_id, self.plan.num_stages
        prev, nxt = self.comm.prev, self.comm.next
        bwd = self.cfg.audit_backward
        act_g, grad_g = (self._dir_groups if self.p2p_mode == "async" else (None, None))
        M = len(self._audit_batch)
        d = rows[self.rank]
        if not hasattr(self, "_audit_rng"):
            seed = self.cfg.monitor_seed
            self._audit_rng = __import__("random").Random(
                int.from_bytes(os.urandom(8), "little") if seed is None else seed * 7919 + self.rank)
        store = dist.distributed_c10d._get_default_store()
        tag = f"tdl_audit/{self.plan.version}/{self.global_step}"
        # my auditees: prev (I am its next stage), and nxt when it is the loss stage
        audit_prev = prev is not None
        audit_next = bwd and nxt is not None and s + 1 == S - 1
        # my auditor: nxt, or prev when I am the loss stage
        my_auditor = nxt if nxt is not None else (prev if bwd and s == S - 1 and prev is not None else None)
        # ---- 1. commitments: running sketches to my auditor before any reveal
        runs_in: Dict[int, torch.Tensor] = {}
        mine = self._gsk_run.get(self.rank) if getattr(self, "_gsk_on", False) else None
        if bwd and mine is not None:
            c_send = [(mine, my_auditor)] if my_auditor is not None else []
            c_recv = []
            for peer, on in ((prev, audit_prev), (nxt, audit_next)):
                if on:
                    runs_in[peer] = torch.empty(M + 1, 2, dtype=torch.float32, device=self.device)
                    c_recv.append((runs_in[peer], peer))
            self._audit_transfer(c_send, c_recv, prev, nxt, act_g, grad_g)

        # ---- 2. reveal: private choices (whether + which micro-batches).  The uniform draw, plus
        # with ``audit_targeted`` the micro-batch whose received output / committed sketch norm stands
        # out (one host read of the scores: the choice needs them)
        tgt_prev = tgt_next = -1
        if self._targeted:
            zs = []
            if audit_prev:
                ys = [self._output_stat(self._audit_inputs[m]) for m in range(M)] if s - 1 >= 0 else None
                zs.append(self._target_scores(ys, runs_in.get(prev)))
            if audit_next:
                zs.append(self._target_scores(None, runs_in.get(nxt)))
            got = [torch.stack([z.max(), z.argmax().float()]) if z is not None else
                   torch.tensor([-1.0, -1.0], device=self.device) for z in zs]
            note_host_sync()
            vals = torch.stack(got).tolist() if got else []
            thr = self.cfg.audit_target_z
            picks = [int(i) if zm > thr else -1 for zm, i in vals]
            if audit_prev:
                tgt_prev = picks.pop(0)
            if audit_next:
                tgt_next = picks.pop(0)
            tl = self.__dict__.setdefault("_target_log", [])
            tl.extend((self.global_step, n, m) for n, m in ((prev, tgt_prev), (nxt, tgt_next)) if m >= 0)

        def choose(extra):
            if self.cfg.audit_prob < 1.0 and self._audit_rng.random() >= self.cfg.audit_prob:
                return [extra] if extra >= 0 else []
            return list(dict.fromkeys([self._audit_rng.randrange(M)] + ([extra] if extra >= 0 else [])))
        ms_prev = choose(tgt_prev) if audit_prev else []
        ms_next = choose(tgt_next) if audit_next else []

        def enc(ms):
            return ",".join(str(m) for m in ms) if ms else "-1"

        def dec(v):
            return [int(t) for t in v.decode().split(",") if int(t) >= 0]
        if audit_prev:
            store.set(f"{tag}/req/{prev}", enc(ms_prev))
            if s - 1 > 0 and bwd:
                store.set(f"{tag}/reqh/{prev}", enc(ms_prev))   # for the stage before prev: dx hash
        if audit_next:
            store.set(f"{tag}/req/{nxt}", enc(ms_next))
        ms_req: List[int] = []
        if my_auditor is not None:
            k = f"{tag}/req/{self.rank}"
            ms_req = dec(store.get(k))
            store.delete_key(k)

        def hsum(ts):
            """Combined hash of several tensors (sum of the 16-bit halves mod 2^16, exact in fp32)."""
            h = hash2(ts[0])
            for t in ts[1:]:
                h = torch.remainder(h + hash2(t), 65536.0)
            return h
        # as the upstream recipient of nxt's input gradient: hash what I received for nxt's audited micro-batches
        if bwd and nxt is not None and s + 1 < S - 1:
            k = f"{tag}/reqh/{nxt}"
            mh = dec(store.get(k))
            store.delete_key(k)
            if mh and all(m in self._audit_recv_dy for m in mh):
                d[SV.D_DXHASH_RECV:SV.D_DXHASH_RECV + 2].copy_(hsum([self._audit_recv_dy[m] for m in mh]))
            else:
                d[SV.D_DXHASH_RECV:SV.D_DXHASH_RECV + 2].fill_(-1.0)
        else:
            d[SV.D_DXHASH_RECV:SV.D_DXHASH_RECV + 2].fill_(-1.0)
        x_send, dx_send = [], []
        if ms_req and s > 0 and s < S - 1:
            x_send = [self._audit_inputs[m].contiguous() for m in ms_req]
            if bwd and all(m in self._audit_sent_dx for m in ms_req):
                dx_send = [self._audit_sent_dx[m].contiguous() for m in ms_req]
            store.set(f"{tag}/shape/{self.rank}", ",".join(str(v) for v in x_send[0].shape))
        # ---- 3. ship (the weights went out before the schedule when ``_audit_early_ship`` ran)
        early = getattr(self, "_early_ship", None)
        self._early_ship = None
        sends, recvs = [], []
        if ms_req:
            if early is None:
                sends.append((st.flat.data, my_auditor))
            sends += [(t, my_auditor) for t in x_send]
            sends += [(t, my_auditor) for t in dx_send]
        mir_p = mir_n = None
        x_prev, dx_prev = [], []
        if audit_prev and ms_prev:
            mir_p = self._audit_mirror(tuple(self.plan.ranges[s - 1]), s - 1)
            if early is None:
                recvs.append((mir_p.flat.data, prev))
            if s - 1 > 0:
                k = f"{tag}/shape/{prev}"
                shape = torch.Size([int(v) for v in store.get(k).decode().split(",")])
                store.delete_key(k)
                x_prev = [torch.empty(shape, dtype=self.dtype, device=self.device) for _ in ms_prev]
                recvs += [(t, prev) for t in x_prev]
                if bwd:
                    dx_prev = [torch.empty(shape, dtype=self.dtype, device=self.device) for _ in ms_prev]
                    recvs += [(t, prev) for t in dx_prev]
        if audit_next and ms_next:
            mir_n = self._audit_mirror(tuple(self.plan.ranges[s + 1]), s + 1)
            if early is None:
                recvs.append((mir_n.flat.data, nxt))
        self._audit_transfer(sends, recvs, prev, nxt, act_g, grad_g)
        if early is not None:
            for w in early[0]:
                w.wait()

        def combine(acc, res):
            if acc is None:
                return res
            (f0, k0, e0), (f1, k1, e1) = acc, res
            return (torch.maximum(f0, f1), torch.bitwise_or(k0.long(), k1.long()).float(), torch.maximum(e0, e1))
        # ---- 4. verify
        if mir_p is not None:
            res = None
            for j, m in enumerate(ms_prev):
                xp = x_prev[j] if x_prev else self._stage_input(self._audit_batch[m], mir_p)
                dy = self._audit_sent_dx.get(m) if bwd else None
                res = combine(res, self._audit_one(mir_p, xp, m, M, y_seen=self._audit_inputs[m], dy=dy,
                                                   dx_seen=dx_prev[j] if dx_prev else None, run=runs_in.get(prev)))
            flag, kind, err = res
            d[SV.D_AUDIT_PREV:SV.D_AUDIT_PREV + 1].copy_(flag)
            d[SV.D_AUDITED_PREV:SV.D_AUDITED_PREV + 1].fill_(1.0)
            d[SV.D_AUDIT_KIND_PREV:SV.D_AUDIT_KIND_PREV + 1].copy_(kind)
            d[SV.D_AUDIT_ERR:SV.D_AUDIT_ERR + 1].copy_(err)
            d[SV.D_WHASH_PREV:SV.D_WHASH_PREV + 2].copy_(hash2(mir_p.flat.data))
            if dx_prev:
                d[SV.D_DXHASH_SHIP:SV.D_DXHASH_SHIP + 2].copy_(hsum(dx_prev))
            else:
                d[SV.D_DXHASH_SHIP:SV.D_DXHASH_SHIP + 2].fill_(-1.0)
        else:
            d[SV.D_WHASH_PREV:SV.D_WHASH_PREV + 2].fill_(-1.0)
            d[SV.D_DXHASH_SHIP:SV.D_DXHASH_SHIP + 2].fill_(-1.0)
        if mir_n is not None:
            res = None
            for m in ms_next:
                labels = self._audit_targets[m].to(self.device, non_blocking=True)
                res = combine(res, self._audit_one(mir_n, self._audit_outputs.get(m), m, M, labels=labels,
                                                   dx_seen=self._audit_recv_dy.get(m), run=runs_in.get(nxt)))
            flag, kind, err = res
            d[SV.D_AUDIT_NEXT:SV.D_AUDIT_NEXT + 1].copy_(flag)
            d[SV.D_AUDITED_NEXT:SV.D_AUDITED_NEXT + 1].fill_(1.0)
            d[SV.D_AUDIT_KIND_NEXT:SV.D_AUDIT_KIND_NEXT + 1].copy_(kind)
            d[SV.D_AUDIT_ERR:SV.D_AUDIT_ERR + 1].copy_(torch.maximum(d[SV.D_AUDIT_ERR:SV.D_AUDIT_ERR + 1], err))
            d[SV.D_WHASH_NEXT:SV.D_WHASH_NEXT + 2].copy_(hash2(mir_n.flat.data))
        else:
            d[SV.D_WHASH_NEXT:SV.D_WHASH_NEXT + 2].fill_(-1.0)
        self._audit_inputs = {}
        self._audit_sent_dx = {}
        self._audit_recv_dy = {}
        self._audit_outputs = {}

    def _note_audit_cost(self, host_s: float, ev):
        a = self.__dict__.setdefault("_audit_cost", {"steps": 0, "host_s": 0.0, "bytes": 0, "events": []})
        a["steps"] += 1
        a["host_s"] += host_s
        if ev is not None:
            a["events"].append(ev)
            if len(a["events"]) > 512:
                del a["events"][:256]

    def audit_summary(self) -> Dict[str, float]:
        """Per-step cost of the recompute audit on this rank (call after a device sync): P2P bytes
        it sent + received (commitments, weights, inputs, gradients), host wall time of the audit
        phase, and device time between its first and last kernel (HIP events)."""
        a = getattr(self, "_audit_cost", None)
        tl = getattr(self, "_target_log", [])
        if not a or not a["steps"]:
            return {"steps": 0, "targeted_extra": len(tl)}
        gpu = [e0.elapsed_time(e1) for e0, e1 in a["events"] if e1.query()]
        return {"steps": a["steps"], "bytes_per_step": a["bytes"] / a["steps"],
                "host_ms_per_step": 1e3 * a["host_s"] / a["steps"],
                "device_ms_per_step": (sum(gpu) / len(gpu)) if gpu else None,
                "targeted_extra": len(tl)}

    def _audit_transfer(self, sends, recvs, prev, nxt, act_g, grad_g):
        """Audit traffic: toward the next stage on the activation communicator, toward the
        previous one on the gradient communicator (async P2P mode; grouped mode: default group),
        as two batched exchanges in the same order on every rank."""
        fwd_s = [(t, r) for t, r in sends if r == nxt]
        fwd_r = [(t, r) for t, r in recvs if r == prev]
        bwd_s = [(t, r) for t, r in sends if r == prev]
        bwd_r = [(t, r) for t, r in recvs if r == nxt]
        a = self.__dict__.setdefault("_audit_cost", {"steps": 0, "host_s": 0.0, "bytes": 0, "events": []})
        a["bytes"] += sum(t.numel() * t.element_size() for t, _ in list(sends) + list(recvs))
        for ss, rr, g in ((fwd_s, fwd_r, act_g), (bwd_s, bwd_r, grad_g)):
            self._note_peers(ss, rr, "dir" if g is not None else "default")
            batched_transfer(ss, rr, group=g)

    def _audit_mirror(self, rng: Tuple[int, int], sid: int) -> Stage:
        """The audited stage's layers on this GPU (weights overwritten by every audit); one mirror
        per audited layer range (the stage before the loss stage audits two stages)."""
        key = (self.plan.version, tuple(rng))
        cache = self.__dict__.setdefault("_mirrors", {})
        if key not in cache:
            for k in [k for k in cache if k[0] != self.plan.version]:
                del cache[k]
            # (its gradient-folding hooks stay: the backward audit recomputes weight gradients on it)
            cache[key] = Stage(self.model, rng, sid, self.plan.num_stages, self.device, self.dtype,
                               {"output_detection": False, "gradient_verification": False, "serialize_streams": True})
        return cache[key]

    def _audit_vectors(self, D: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Per-node (failed-check bitmask, audited) from the digest, identical on every rank: a
        stage's verdict sits in the row of its auditor (the next stage of its pipeline replica; the
        loss stage's in its predecessor's ``*_NEXT`` slots), plus the hash cross-checks — the
        weights its auditor received vs its own post-update commitment, and the input gradient it
        shipped to its auditor vs what the upstream stage received."""
        N = D.shape[0]
        kind = torch.zeros(N, dtype=torch.float32, device=D.device)
        done = torch.zeros_like(kind)
        bwd = self.cfg.audit_backward
        for idx in self._replica_orders():
            n = idx.numel()
            if n < 2:
                continue
            a, p = idx[1:], idx[:-1]
            kind[p] = D[a, SV.D_AUDIT_KIND_PREV] + (D[a, SV.D_AUDIT_PREV] > 0).float() * \
                (D[a, SV.D_AUDIT_KIND_PREV] <= 0).float() * SV.AK_FWD
            done[p] = D[a, SV.D_AUDITED_PREV]
            if self.distributed:
                wh_c, wh_s = D[p, SV.D_WHASH:SV.D_WHASH + 2], D[a, SV.D_WHASH_PREV:SV.D_WHASH_PREV + 2]
                both = ((wh_c[:, 0] >= 0) & (wh_s[:, 0] >= 0)).float()
                kind[p] += both * (wh_c != wh_s).any(1).float() * SV.AK_WHASH
                if n >= 3:
                    # stage j (1 <= j <= n-2) shipped its dx to idx[j+1]; idx[j-1] received it
                    q = idx[1:-1]
                    recv, ship = D[idx[:-2], SV.D_DXHASH_RECV:SV.D_DXHASH_RECV + 2], \
                        D[idx[2:], SV.D_DXHASH_SHIP:SV.D_DXHASH_SHIP + 2]
                    both = ((recv[:, 0] >= 0) & (ship[:, 0] >= 0)).float()
                    kind[q] += both * (recv != ship).any(1).float() * SV.AK_DXHASH
            if bwd:
                L, A = idx[-1], idx[-2]
                kind[L] = D[A, SV.D_AUDIT_KIND_NEXT]
                done[L] = D[A, SV.D_AUDITED_NEXT]
                if self.distributed:
                    wh_c, wh_s = D[L, SV.D_WHASH:SV.D_WHASH + 2], D[A, SV.D_WHASH_NEXT:SV.D_WHASH_NEXT + 2]
                    both = float(1.0) * ((wh_c[0] >= 0) & (wh_s[0] >= 0)).float()
                    kind[L] += both * (wh_c != wh_s).any().float() * SV.AK_WHASH
        return kind, done

    def _gsk_mismatch(self, D: torch.Tensor) -> torch.Tensor:
        """Per-node 1.0 where the applied gradient's sketch differs from the committed sum of the
        stage's per-micro-batch contributions (a gradient rewritten after the backward)."""
        from ..security.grad_audit import K_SKETCH
        app = D[:, SV.D_GSK_APP:SV.D_GSK_APP + K_SKETCH]
        com = D[:, SV.D_GSK_BWD:SV.D_GSK_BWD + K_SKETCH]
        on = (D[:, SV.D_GSK_ON] > 0).float()
        scale = torch.maximum(com.abs().amax(1), app.abs().amax(1)).clamp_min(1e-20)
        err = torch.nan_to_num((app - com).abs().amax(1) / scale, nan=1e30, posinf=1e30)
        bad = on * (err > 1e-3).float()
        # the tied weight: every member must apply the sum of the members' own contributions
        ton = (D[:, SV.D_TSK_ON] > 0).float()
        pre, tapp = D[:, SV.D_TSK_PRE:SV.D_TSK_PRE + K_SKETCH], D[:, SV.D_TSK_APP:SV.D_TSK_APP + K_SKETCH]
        for idx in self._replica_orders():
            t = ton[idx]
            exp = (pre[idx] * t[:, None]).sum(0, keepdim=True)
            sc = torch.maximum(exp.abs().amax(), tapp[idx].abs().amax(1)).clamp_min(1e-20)
            e = torch.nan_to_num((tapp[idx] - exp).abs().amax(1) / sc, nan=1e30, posinf=1e30)
            bad[idx] = torch.maximum(bad[idx], t * (t.sum() >= 2).float() * (e > 1e-3).float())
        return bad

    # ================================================================== integrity + attribution
    @torch.no_grad()
    def _integrity_flag(self, st: Stage) -> torch.Tensor:
        """1.0 when the stage's compute weights differ from the checksum taken right after its last
        optimizer step (a write outside the optimizer), else 0.0 — device-side, no sync."""
        cur = st.__dict__.pop("_early_checksum", None)
        if cur is None:
            cur = dstats.checksum(st.flat.data)
        st._cur_checksum = cur
        # a write between the start of the previous step and its update (during its forward /
        # backward: ADVICE r3) was seen by that step's tail re-check and is reported now
        tail = st.__dict__.pop("_tail_flag", None)
        ref = getattr(st, "param_checksum", None)
        if ref is None:  # first step / freshly (re)built or reloaded stage: nothing to compare yet
            st.param_checksum = cur
            return torch.zeros(1, dtype=torch.float32, device=st.device)
        flag = (cur != ref).any().float().reshape(1)
        return flag if tail is None else torch.maximum(flag, tail)

    def _replica_orders(self) -> List[torch.Tensor]:
        key = (self.plan.version, self.dp)
        if getattr(self, "_orders_key", None) != key:
            base = self.replica * self.pp
            self._orders = [torch.tensor([d * self.pp + (r - base) for r in self.plan.ranks], dtype=torch.long,
                                         device=self.device) for d in range(self.dp)]
            self._orders_key = key
        return self._orders

    def _attribute(self, D: torch.Tensor) -> torch.Tensor:
        """Per-node (blame, evidence) for this step, identical on every rank (device, from the
        all-gathered D); ``evidence[n]`` = 1 when n's pipeline replica saw a tampered forward.

        In a pipeline an anomaly echoes: tampered activations of stage s make every later stage's
        output (and, through backward, every stage's gradients) look anomalous too.  Blame goes to
        (a) any stage whose weights failed the integrity check, (b) the EARLIEST stage of each
        pipeline replica with an output anomaly, and (c) gradient anomalies only when the replica
        shows no output / integrity evidence (gradient poisoning does not propagate)."""
        of, gf, pf = D[:, SV.D_OUT_FLAG], D[:, SV.D_GRAD_FLAG], D[:, SV.D_PARAM_FLAG]
        oz = D[:, SV.D_OUT_Z]
        blame = torch.zeros_like(of)
        evidence = torch.zeros_like(of)
        self.t_taint.copy_(torch.maximum(self.t_taint, (pf > 0).float()))
        audited = getattr(self, "_audit_now", False)
        akind = torch.zeros_like(of)
        if audited:
            akind, _ = self._audit_vectors(D)
        abad = (akind > 0).float()
        # applied gradient != committed backward contributions: rewritten after the backward
        gbad = self._gsk_mismatch(D) if self.cfg.audit and self.cfg.audit_backward else torch.zeros_like(of)
        # proof of tampering (not a statistic): compromises at once (compromise_on_proof)
        self._proof = torch.maximum(torch.maximum((pf > 0).float(), abad), gbad)
        self._proof_kind = akind + gbad * 32.0
        stat_blame = 0.0 if (audited and self.cfg.audit_backward) else 1.0
        for r, idx in enumerate(self._replica_orders()):
            o, g, p = of[idx], gf[idx], pf[idx]
            taint = self.t_taint[idx]
            ev = torch.maximum(o.max(), p.max())
            if audited:
                # deterministic attribution: a tampered forward is blamed only on a recompute
                # mismatch (its own stage, never the downstream echoes) or a failed weight-integrity
                # check; output z-scores do not blame.  Gradient anomalies count only in a replica
                # without such evidence (gradient poisoning does not propagate, tampering does)
                # with the backward audit, gradient z-scores no longer blame either: the
                # deterministic gradient checks (recomputed contribution, applied-vs-committed
                # sketch) do; the statistics still quarantine the update and feed the trust metrics
                a = abad[idx]
                ev = torch.maximum(p.max(), a.max())
                b = torch.maximum(torch.maximum(p, a), g * (1.0 - ev) * stat_blame)
                o = a   # "forward anomaly" below = a recompute mismatch
            elif self.cfg.attribute_flags:
                # earliest anomalous stage; a stage with tampered (integrity-failed, not yet
                # restored) weights counts as anomalous, so the output echoes it causes downstream
                # are neither blamed nor skip the step (its own flag already compromised it)
                if self.cfg.soft_output_z > 0:
                    # a replica with an output flag: softly anomalous earlier stages count too
                    soft = (oz[idx] > self.cfg.soft_output_z).float() * o.max()
                    o = torch.maximum(o, soft)
                a = torch.maximum(o, taint)
                head = (torch.cumsum(a, 0) == 1).float() * a
                first = head * o * (1.0 - taint)
                b = torch.maximum(torch.maximum(p, first), g * (1.0 - ev))
                ev = torch.maximum(p.max(), (head * o * (1.0 - taint)).max())
            else:
                b = torch.maximum(torch.maximum(o, g), p)
            n = idx.numel()
            if self.cfg.global_event_fraction > 0 and n >= 3:
                # pipeline-wide gradient anomaly (every stage's norm jumps together in a loss spike):
                # skip the update, blame nobody, and keep output / gradient blame off for a grace
                # window; integrity (parameter) evidence is never suppressed
                # (with an output anomaly in the replica the gradient flags are echoes of a tampered
                # forward instead, attributed to its earliest stage above)
                glob = (g.sum() >= max(2.0, math.ceil(self.cfg.global_event_fraction * n))).float() * (1.0 - o.max())
                gr = self.t_grace[r:r + 1]
                gr.copy_(torch.maximum(gr - 1.0, torch.zeros_like(gr)) * (1.0 - glob)
                         + glob * float(self.cfg.global_event_grace))
                quiet = torch.maximum(glob, (gr > 0).float())
                if audited:
                    # a recompute mismatch is proof, not a statistic: never quieted (a grace window
                    # opened by an earlier loss spike let tampered steps through in r4's first runs)
                    b = torch.maximum(torch.maximum(p, o), b * (1.0 - quiet))
                    ev = torch.maximum(torch.maximum(p.max(), o.max()), glob)
                else:
                    b = torch.maximum(p, b * (1.0 - quiet))
                    ev = torch.maximum(torch.maximum(p.max(), o.max() * (1.0 - quiet)), glob)
            gb = gbad[idx]
            blame[idx] = torch.maximum(b, gb)
            # a gradient rewritten after the backward skips that stage's update (it does not echo)
            evidence[idx] = torch.maximum(ev.expand(n), gb)
        return blame, evidence

    # ================================================================== heartbeat -> OFFLINE
    def _apply_offline(self, D: torch.Tensor):
        """A node is OFFLINE while any rank's watchdog reports it silent (union of the all-gathered
        bitmasks, identical on every rank); a node no rank reports any more goes RECOVERING.
        Device-side, so every rank's trust state moves identically without a host sync."""
        N = self.num_nodes
        bits = D[:, SV.D_OFFLINE_MASK].to(torch.int64)
        shifts = torch.arange(N, device=self.device, dtype=torch.int64)
        off = ((bits[:, None] >> shifts[None, :]) & 1).amax(0).to(torch.bool)
        OFF = STATUS_CODES[NodeStatus.OFFLINE]
        was_off = self.t_status == OFF
        self.t_status.copy_(torch.where(off, torch.full_like(self.t_status, OFF),
                                        torch.where(was_off, torch.full_like(self.t_status,
                                                                             STATUS_CODES[NodeStatus.RECOVERING]),
                                                    self.t_status)))

    def close(self):
        if self.heartbeat is not None:
            self.heartbeat.stop()
            self.heartbeat = None

    # ================================================================== data parallelism (pipeline replicas)
    def all_ranks(self) -> List[int]:
        """Every rank holding a stage: the plan's ranks in each replica."""
        if self.dp == 1:
            return list(self.plan.ranks)
        base = self.replica * self.pp
        return [d * self.pp + (r - base) for d in range(self.dp) for r in self.plan.ranks]

    def last_ranks(self) -> List[int]:
        base = self.replica * self.pp
        return [d * self.pp + (self.plan.ranks[-1] - base) for d in range(self.dp)]

    def _dp_group_ranks(self) -> List[int]:
        pos = self.rank % self.pp
        return [d * self.pp + pos for d in range(self.dp)]

    def _dp_aggregate(self, D: torch.Tensor, evidence: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Byzantine-robust gradient mean across this stage's replicas, all on device.

        A replica is left out when its own verifier flagged the gradient, it produced non-finite
        values, its node is COMPROMISED, or (>= 3 replicas) its gradient norm is an outlier
        against the replicas' median.  Each rank scales its flat gradient by ok / n_ok and the
        replicas all-reduce (sum) -> mean of the trusted replicas; if none is trusted the step is
        skipped on every replica (weights stay identical).  Returns the global sum of squares of the
        aggregated gradient (for clipping), from one extra scalar all-reduce."""
        st = self.my_stage()
        ranks = self._dp_group_ranks()
        idx = self._index_tensor(ranks)
        rows = D[idx]
        bad = torch.maximum(rows[:, SV.D_GRAD_FLAG], (rows[:, SV.D_NONFINITE] > 0).float())
        bad = torch.maximum(bad, (self.t_status[idx] == STATUS_CODES[NodeStatus.COMPROMISED]).float())
        if evidence is not None:
            bad = torch.maximum(bad, evidence[idx])  # the replica's forward was tampered
        if len(ranks) >= 3:
            norms = rows[:, SV.D_GRAD_L2]
            med = norms.median()
            ratio = norms / torch.clamp(med, min=1e-30)
            tau = float(self.cfg.outlier_ratio)
            bad = torch.maximum(bad, ((ratio > tau) | (ratio < 1.0 / tau)).float())
            if st is not None and self.cfg.robust_aggregation:
                bad = torch.maximum(bad, self._dp_direction_outliers(st, len(ranks), bad[ranks.index(self.rank)]))
        if not self.cfg.robust_aggregation:
            bad = torch.zeros_like(bad)
        ok = 1.0 - bad
        n_ok = ok.sum()
        me = ranks.index(self.rank)
        w = ok[me] / torch.clamp(n_ok, min=1.0)
        if st is not None:
            st.flat.grad.mul_(w)
            # an excluded replica contributes exactly zero: NaN/Inf * 0 is NaN, so clear it outright
            st.flat.grad.masked_fill_(w <= 0, 0.0)
            dist.all_reduce(st.flat.grad, group=self.dp_group)
            st.verifier.ctrl[1:2].copy_((n_ok < 0.5).float().reshape(1))
            sq = st.clip_sumsq(st.flat.grad).reshape(1)
        else:
            sq = torch.zeros(1, device=self.device)
        self._dp_excluded = bad
        dist.all_reduce(sq)
        return (sq / self.dp).reshape(())

    def _dp_direction_outliers(self, st: Stage, n: int, bad_me: torch.Tensor) -> torch.Tensor:
        """Cross-replica direction check (the reference's ``detect_byzantine_behavior`` Gram-matrix
        idea, attack_detector.py:143-162, on a sketch): every replica takes the same strided 1/64
        sample of its flat gradient, one small all-reduce sums the unit-normalised samples of the
        replicas not already excluded, and each replica's cosine to the SUM OF THE OTHERS is
        all-gathered.  A replica pointing against its peers (a sign
        flip, which no per-replica statistic sees) is an outlier: cosine < 0 and more than
        ``direction_margin`` below the replicas' median.  Device-side, no host sync."""
        g = st.flat.grad
        if getattr(self, "_dp_sidx", None) is None or self._dp_sidx.device != g.device:
            self._dp_sidx = torch.arange(0, g.numel(), 64, device=g.device)
        sub = torch.nan_to_num(g.index_select(0, self._dp_sidx), nan=0.0, posinf=0.0, neginf=0.0)
        # unit directions, replicas already excluded (flag / non-finite / norm outlier) left out of
        # the reference: a x50 replica must not define "the others' direction"
        unit = sub / torch.clamp(sub.norm(), min=1e-30)
        contrib = unit * (1.0 - bad_me)
        tot = contrib.clone()
        dist.all_reduce(tot, group=self.dp_group)
        others = tot - contrib
        cos = ((unit * others).sum() / torch.clamp(others.norm(), min=1e-30)).reshape(1)
        allc = [torch.zeros_like(cos) for _ in range(n)]
        dist.all_gather(allc, cos, group=self.dp_group)
        c = torch.cat(allc)
        self._dp_cos = c
        return ((c < 0) & (c < c.median() - float(self.cfg.direction_margin))).float()

    @torch.no_grad()
    def _audit_params(self):
        """Cross-replica weight audit: replicas must hold bit-identical fp32 master weights.  A
        replica whose digest (float64 sum, sum of squares) differs from the majority of its stage
        position was tampered with (parameter perturbation / model poisoning): every rank sees the
        same all-gathered digests, so every rank records it and marks the node compromised in the
        device trust state identically; the stage's replicas then re-synchronise (fp32 master and
        AdamW moments broadcast from a majority member).  One small host read every few steps."""
        st = self.my_stage()
        if st is not None:
            m = st.flat.master.double()
            dg = torch.stack([m.sum(), (m * m).sum()])
        else:
            dg = torch.zeros(2, dtype=torch.float64, device=self.device)
        G = all_gather_rows(dg, self.world)
        note_host_sync()
        G = G.cpu()
        my_pos = self.rank % self.pp
        for pos in range(self.pp):
            ranks = [d * self.pp + pos for d in range(self.dp)]
            rows = [tuple(G[r].tolist()) for r in ranks]
            counts: Dict[tuple, int] = {}
            for r in rows:
                counts[r] = counts.get(r, 0) + 1
            majority, votes = max(counts.items(), key=lambda kv: kv[1])
            divergent = [ranks[i] for i, r in enumerate(rows) if r != majority]
            if not divergent:
                continue
            src = ranks[rows.index(majority)] if votes * 2 > len(ranks) else None
            rec = {"step": self.global_step, "timestamp": time.time(), "attack_type": "model_poisoning",
                   "divergent_nodes": divergent, "resync_from": src, "stage_position": pos}
            self.dp_audits.append(rec)
            logger.warning("parameter audit: replicas %s diverge from the majority (resync from %s)", divergent, src)
            for n in divergent:
                self.attack_history.append({"node_id": n, "timestamp": rec["timestamp"], "step": self.global_step,
                                            "attack_type": "model_poisoning", "ground_truth": None})
                self.trust.mark_compromised(n, "model_poisoning")
                self.t_values[n] = 0.1
                self.t_status[n] = STATUS_CODES[NodeStatus.COMPROMISED]
            if pos == my_pos and src is not None and st is not None:
                for buf in st.flat.optimizer_state_tensors():
                    dist.broadcast(buf, src, group=self.dp_group)
                if st.flat.data is not st.flat.master:
                    st.flat.data.copy_(st.flat.master)
                st.param_checksum = None

    # ================================================================== host-side report processing
    def flush(self) -> Optional[float]:
        self._consume_reports(upto=None)
        return self.last_loss

    def _consume_reports(self, upto: Optional[int]):
        while self._pending and (upto is None or self._pending[0][0] <= upto):
            step, epoch, host, ev, truth, lasts = self._pending.popleft()
            note_host_sync()
            if ev is not None:
                ev.synchronize()
            self._process_report(step, epoch, host, truth, lasts)

    def _process_report(self, step: int, epoch: int, host: torch.Tensor, truth: Dict[int, bool],
                        loss_ranks: Optional[List[int]] = None):
        N = self.num_nodes
        D = host[: N * SV.DIGEST].view(N, SV.DIGEST).tolist()
        values = host[N * SV.DIGEST: N * SV.DIGEST + N].tolist()
        statuses = [int(v) for v in host[N * SV.DIGEST + N:N * SV.DIGEST + 2 * N].tolist()]
        blamed = [v > 0 for v in host[N * SV.DIGEST + 2 * N:N * SV.DIGEST + 3 * N].tolist()]
        audit_kind = [int(v) for v in host[N * SV.DIGEST + 3 * N:N * SV.DIGEST + 4 * N].tolist()]
        audit_bad = [k > 0 for k in audit_kind]
        present = set(self.all_ranks())
        # the loss stages of the plan the step ran under (a re-shard decided by an earlier report
        # may have moved the loss stage since)
        lasts = [n for n in (loss_ranks if loss_ranks is not None else self.last_ranks()) if D[n][SV.D_PRESENT] > 0]
        self.last_loss = sum(D[n][SV.D_LOSS] for n in lasts) / len(lasts) if lasts else None
        detections = []
        for n in range(N):
            row = D[n]
            if n not in present or row[SV.D_PRESENT] <= 0:
                continue
            gt = bool(row[SV.D_ATTACK_TRUTH] > 0)
            out_flag, grad_flag = row[SV.D_OUT_FLAG] > 0, row[SV.D_GRAD_FLAG] > 0
            param_flag = row[SV.D_PARAM_FLAG] > 0
            flagged = blamed[n]
            if flagged:
                kind = self._evidence_kind(param_flag, audit_kind[n], out_flag)
                rec = {"node_id": n, "timestamp": time.time(), "step": step, "attack_type": kind,
                       "output_stats": {"mean": row[SV.D_OUT_MEAN], "std": row[SV.D_OUT_STD],
                                        "z": row[SV.D_OUT_Z]},
                       "gradient_stats": {"norm_l2": row[SV.D_GRAD_L2], "z": row[SV.D_GRAD_Z],
                                          "cosine": row[SV.D_GRAD_COS]},
                       "audit_kind": audit_kind[n], "ground_truth": gt}
                self.attack_history.append(rec)
                self.trust.attack_history[n].append({"timestamp": rec["timestamp"], "step": step,
                                                     "attack_type": kind,
                                                     "previous_trust": self.trust.get_trust_score(n)})
                detections.append(n)
            if self.detector is not None:
                ds = self.detector.detection_stats
                if flagged:
                    ds["total_detections"] += 1
                    k = self._evidence_kind(param_flag, audit_kind[n], out_flag)
                    k = {"output_tampering": "byzantine", "output_anomaly": "byzantine",
                         "gradient_tampering": "byzantine"}.get(k, k)
                    ds["attack_types"][k] = ds["attack_types"].get(k, 0) + 1
                key = ("true_positives" if gt else "false_positives") if flagged else \
                      ("false_negatives" if gt else "true_negatives")
                ds[key] += 1
            if self.attacker is not None and hasattr(self.attacker, "record_detection"):
                self.attacker.record_detection(n, step, flagged, gt)
        metrics = [row[SV.D_METRICS:SV.D_METRICS + 6] for row in D]
        prev_status = {n: self.trust.get_node_status(n) for n in range(N)}
        self.trust.ingest_device_update([values[n] for n in range(N)], [statuses[n] for n in range(N)], metrics,
                                        update_counts=None)
        if detections:
            self.state_flags["under_attack"] = True
        if self.metrics is not None:
            self.metrics.collect_batch_metrics({
                "loss": self.last_loss, "step": step, "epoch": epoch,
                "trust_scores": {i: values[i] for i in range(N)},
                "detections": detections, "grad_norm": [D[n][SV.D_GRAD_L2] for n in range(N)],
                "step_time": self._step_time})
        OFF = STATUS_CODES[NodeStatus.OFFLINE]
        for n in range(N):
            if (statuses[n] == OFF) != (prev_status.get(n) == NodeStatus.OFFLINE):
                self.node_events.append({"node_id": n, "step": step, "timestamp": time.time(),
                                         "event": "offline" if statuses[n] == OFF else "online"})
        self._commit_shadows(step, blamed, statuses)
        newly = [n for n in range(N) if n in present and statuses[n] == STATUS_CODES[NodeStatus.COMPROMISED]
                 and prev_status.get(n) != NodeStatus.COMPROMISED]
        newly += [n for n in range(N) if n in present and statuses[n] == STATUS_CODES[NodeStatus.COMPROMISED]
                  and n not in newly and n in detections]
        if newly and self.cfg.reassign:
            self.reassign(sorted(set(newly)), step)
        # runtime metrics for the next digest (latency s, utilization, error, uptime)
        util = 1.0 - (self._comm_wait / self._step_time) if self._step_time > 0 else 0.0
        for n in range(N):
            self._host_metrics[n] = [self._comm_wait, max(0.0, min(1.0, util)), 0.0, 1.0]

    def _evidence_kind(self, param_flag: bool, kind: int, out_flag: bool) -> str:
        """Attack record type from the evidence behind a blame (audit bitmask AK_*, 32 = applied
        gradient differs from the committed backward)."""
        if param_flag or kind & SV.AK_WHASH:
            return "model_poisoning"
        if kind & SV.AK_FWD:
            return "output_tampering"
        if kind & (SV.AK_DX | SV.AK_DXHASH):
            return "gradient_tampering"
        if kind & (SV.AK_DW | 32):
            return "gradient_poisoning"
        return "output_anomaly" if out_flag and not self.cfg.audit else "gradient_poisoning"

    # ================================================================== re-sharding (task reassignment)
    def estimate_migration_time(self, layer_numel: int, links: int = 1, plan: Optional[PlacementPlan] = None) -> float:
        """Predicted wall time of a re-shard that moves ``layer_numel`` parameters to ``plan``.

        transfer: fp32 master + 2 AdamW moments (12 B/param) over ``links`` peer links at the per-link
        throughput MEASURED on this job's own bulk transfers (shadow snapshots, earlier migrations:
        ``comm.LinkMeter``; before the first one, a prior of one xGMI link, ~150 GB/s; gloo 2 GB/s);
        pack + unpack: the rank's share of the packed state, at the device copy rate;
        rebuild: stage modules, flat buffers and verifiers of the new plan, at the per-parameter
        rates measured when this engine built its stages (``_build_times``) and refitted from every
        re-shard's measured phases (``_migrate_phases``);
        groups: communicator set-up of the new plan (cached groups cost nothing).
        The reference uses a fixed 1 GiB/s + 2 s (distributed_trainer.py:354-365)."""
        bw = self.link_meter.bytes_per_s() * max(1, links)
        cal = self._reshard_calibration()
        if plan is None:
            plan = self.plan
        mine = [li for li in range(self.num_layers) if not self.distributed or plan.owner_of_layer(li) == self.rank]
        params = sum(self._layer_numel(li) for li in mine)
        local_bytes = sum(self._packed_numel(li) * 4 for li in mine)
        fresh = layer_numel if self.distributed else 0   # layers new to a rank are deep-copied there
        one_device = not self.distributed and len({st.device for st in self.stages.values()}) <= 1
        xfer = 0.0 if one_device else layer_numel * 12 / bw   # local, one GPU: the state stays in HBM
        est = (xfer
               + local_bytes * cal["copy_s_per_byte"]
               + params * cal["flatten_s_per_param"] + fresh * cal["materialize_s_per_param"]
               + cal["groups_s"])
        return est

    def _reshard_calibration(self) -> Dict[str, float]:
        """Rates behind ``estimate_migration_time``: the median over this engine's initial build and
        every re-shard measured so far (``_reshard_samples``; a median keeps one slow outlier, e.g.
        an allocator flush during a rebuild, from skewing the next prediction)."""
        bt = getattr(self, "_init_build_times", None) or getattr(self, "_build_times", {})
        mat_rate = bt.get("materialize_s", 0.0) / max(1, bt.get("materialized_params", 1))
        flat = [bt.get("flatten_s", 0.0) / max(1, bt.get("flattened_params", 1))]
        copy = [1.0 / (600e9 if self.device.type == "cuda" else 4e9)]   # pack + unpack prior
        groups = [0.0]
        for ph in getattr(self, "_reshard_samples", []):
            if ph.get("local_bytes"):
                copy.append((ph["pack_s"] + ph["unpack_s"]) / ph["local_bytes"])
            if ph.get("flattened_params"):
                flat.append(max(0.0, ph["rebuild_s"] - ph["materialized_params"] * mat_rate) / ph["flattened_params"])
            groups.append(ph.get("groups_s", 0.0))
        med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
        return {"copy_s_per_byte": med(copy), "flatten_s_per_param": med(flat),
                "materialize_s_per_param": mat_rate, "groups_s": med(groups)}

    def reassign(self, compromised: Sequence[int], step: Optional[int] = None):
        """Exclude ``compromised`` nodes and re-partition every layer over the remaining trusted
        ones, migrating weights + optimizer state (distributed_trainer.py:324-380, made real)."""
        if self.dp > 1:
            # replicas keep identical layouts; a compromised replica member is excluded from the
            # gradient mean (robust aggregation) and re-synchronised by the parameter audit instead
            logger.warning("DP=%d: nodes %s excluded from aggregation (no re-shard)", self.dp, list(compromised))
            return
        attempts = sum(1 for r in self.reassignment_history if set(r["from_nodes"]) & set(compromised))
        if attempts >= self.cfg.max_reassignment_attempts:
            logger.warning("max reassignment attempts reached for %s", compromised)
            return
        keep = [r for r in self.plan.ranks if r not in compromised]
        keep = [r for r in keep if self.trust.can_assign_task(r) or r not in compromised]
        if len(keep) < max(1, self.cfg.min_stages):
            logger.error("No trusted nodes available for reassignment")
            return
        keep = keep[: self.num_layers]
        new_plan = make_plan(self.costs, keep, self.plan.version + 1, self.cfg.balanced_partition)
        if self.distributed:
            # one decision for everyone: rank 0's plan is broadcast (every rank computed it from the
            # same all-gathered report, but floats / trust state must not be able to split the job)
            new_plan = PlacementPlan.from_list(broadcast_ints(new_plan.to_list() if self.rank == 0 else None, 0,
                                                              self.device))
        # a compromised stage's layers never come from its own memory: from a committed shadow held by
        # a trusted holder whose copy verifies, else from the initial weights
        verified = self._verify_shadows() if self._shadow_meta else {}
        sources = {c: self._shadow_source(c, compromised, verified) for c in compromised}
        restored = {c: self._shadow_meta[c][0] for c in compromised if sources[c] is not None}
        fresh = [c for c in compromised if sources[c] is None]
        if fresh:
            logger.warning("no verified shadow for %s: their layers restart from the initial weights", fresh)
        to_move = sum(self._layer_numel(li) for li in range(self.num_layers)
                      if self.plan.owner_of_layer(li) != new_plan.owner_of_layer(li) or
                      any(self.plan.owner_of_layer(li) == c for c in compromised))
        predicted = self.estimate_migration_time(to_move, plan=new_plan)   # before the move: a prediction
        t0 = time.perf_counter()
        moved = self._migrate(new_plan, restore={c: sources[c] for c in restored}, fresh=fresh)
        dt = time.perf_counter() - t0
        self.excluded = sorted(set(self.excluded) | set(compromised))
        for c in compromised:     # the tampered weights now live nowhere (restored or re-placed)
            if c < self.t_taint.numel():
                self.t_taint[c] = 0.0
        to_nodes = sorted({new_plan.owner_of_layer(li) for li in range(self.num_layers)
                           if self._old_owner.get(li) in compromised})
        rec = {"from_node": compromised[0], "from_nodes": list(compromised), "to_node": to_nodes[0] if to_nodes else None,
               "to_nodes": to_nodes, "timestamp": time.time(), "migration_time": dt,
               "estimated_migration_time": predicted,
               "phases": {k: (round(v, 6) if isinstance(v, float) else v) for k, v in self._migrate_phases.items()},
               "moved_params": moved, "step": step if step is not None else self.global_step,
               "restored_from_shadow": restored,
               "restored_from_initial": fresh,
               "shadow_holders": {c: sources[c] for c in restored},
               "plan": new_plan.describe()}
        self.reassignment_history.append(rec)
        logger.warning("Reassigned tasks from %s -> %s in %.3fs; new plan %s", compromised, to_nodes, dt,
                       new_plan.describe())

    def _layer_numel(self, li: int) -> int:
        return sum(p.numel() for p in self.layers[li].parameters())

    def _pack_layer(self, st: Stage, li: int) -> torch.Tensor:
        parts = []
        a, _ = st.layer_range
        mod = st.module[li - a]
        pidx = {id(p): i for i, p in enumerate(st.flat.params)}
        for name, p in mod.named_parameters(remove_duplicate=False):
            i = pidx[id(p)]
            for buf in (st.flat.master, st.flat.exp_avg, st.flat.exp_avg_sq):
                parts.append(st.flat.view(buf, i).reshape(-1).float())
        for name, b in mod.named_buffers():
            parts.append(b.detach().reshape(-1).float())
        return torch.cat(parts) if parts else torch.zeros(0, device=st.device)

    def _pack_initial(self, li: int, device) -> torch.Tensor:
        """Layer ``li`` in the migration format from the host model (initial weights, zero AdamW
        moments): the source of last resort for a compromised stage with no verified shadow."""
        parts = []
        for name, p in self.layers[li].named_parameters(remove_duplicate=False):
            v = p.detach().reshape(-1).float()
            parts += [v, torch.zeros_like(v), torch.zeros_like(v)]
        for name, b in self.layers[li].named_buffers():
            parts.append(b.detach().reshape(-1).float())
        return torch.cat(parts).to(device) if parts else torch.zeros(0, device=device)

    def _packed_numel(self, li: int) -> int:
        layer = self.layers[li]
        n = 3 * sum(p.numel() for _, p in layer.named_parameters(remove_duplicate=False))
        n += sum(b.numel() for _, b in layer.named_buffers())
        return n

    def _unpack_into(self, st: Stage, li: int, vec: torch.Tensor):
        a, _ = st.layer_range
        mod = st.module[li - a]
        pidx = {id(p): i for i, p in enumerate(st.flat.params)}
        off = 0
        vec = vec.to(st.device)
        for name, p in mod.named_parameters(remove_duplicate=False):
            i = pidx[id(p)]
            n = p.numel()
            for buf in (st.flat.master, st.flat.exp_avg, st.flat.exp_avg_sq):
                st.flat.view(buf, i).reshape(-1).copy_(vec[off:off + n])
                off += n
        for name, b in mod.named_buffers():
            n = b.numel()
            b.copy_(vec[off:off + n].view(b.shape).to(b.dtype))
            off += n

    def _migrate(self, new_plan: PlacementPlan, restore: Optional[Dict[int, int]] = None,
                 fresh: Sequence[int] = ()) -> int:
        """Move every layer to its new owner.  Layers of the nodes in ``restore`` (owner -> serving
        holder) come from their last committed shadow snapshot, those of the nodes in ``fresh``
        from the initial weights (built by the new owner from the host model) — never from the
        compromised node itself.

        Phases (timed into ``self._migrate_phases``, seconds, device-synchronised at each boundary):
        pack (fp32 master + moments + buffers of every layer leaving or staying, one device vector per
        layer), transfer (P2P over xGMI; local mode: none, the vectors stay in HBM), rebuild (stage
        modules re-used where this rank already holds the layer, else deep-copied; flat buffers,
        verifiers, hooks), groups (communicators of the new plan, cached by member set), unpack."""
        old_plan = self.plan
        self._old_owner = {li: old_plan.owner_of_layer(li) for li in range(self.num_layers)}
        from_shadow: Dict[int, int] = {}     # layer -> holder rank serving it from a shadow
        for c, h in (restore or {}).items():
            a, b = self._shadow_meta[c][1]
            for li in range(a, b):
                from_shadow[li] = h
        from_init = {li for c in fresh for li in range(self.num_layers) if old_plan.owner_of_layer(li) == c}
        step_count = next(iter(self.stages.values())).flat.step_count if self.stages else 0
        packed: Dict[int, torch.Tensor] = {}
        moved = 0
        ph: Dict[str, float] = {}
        self._sync_all()
        t0 = time.perf_counter()
        xfer_bytes = 0
        if self.distributed:
            sends, recvs = [], []
            for li in range(self.num_layers):
                src, dst = old_plan.owner_of_layer(li), new_plan.owner_of_layer(li)
                if li in from_shadow:
                    src = from_shadow[li]
                if li in from_init:
                    if dst == self.rank:
                        packed[li] = self._pack_initial(li, self.device)
                    moved += self._layer_numel(li)
                    continue
                if src == self.rank:
                    vec = (self._shadow_slice(li) if li in from_shadow
                           else self._pack_layer(self.stages[self.rank], li))
                    if dst == self.rank:
                        packed[li] = vec
                    else:
                        sends.append((vec, dst))
                        xfer_bytes += vec.numel() * 4
                if dst == self.rank and src != self.rank:
                    buf = torch.empty(self._packed_numel(li), dtype=torch.float32, device=self.device)
                    recvs.append((buf, src))
                    packed[li] = buf
                if src != dst:
                    moved += self._layer_numel(li)
            self._sync_all()
            t1 = time.perf_counter()
            self._note_peers(sends, recvs)
            batched_transfer(sends, recvs, meter=self.link_meter)
            step_t = torch.tensor([float(step_count)], device=self.device)
            dist.all_reduce(step_t, op=dist.ReduceOp.MAX)
            note_host_sync()
            step_count = int(step_t.item())
        else:
            # every stage is local: the packed vectors stay on the device (no host round trip)
            for li in range(self.num_layers):
                src, dst = old_plan.owner_of_layer(li), new_plan.owner_of_layer(li)
                if li in from_init:
                    packed[li] = self._pack_initial(li, self.stages[src].device)
                else:
                    packed[li] = (self._shadow_slice(li) if li in from_shadow
                                  else self._pack_layer(self.stages[src], li))
                if src != dst:
                    moved += self._layer_numel(li)
            self._sync_all()
            t1 = time.perf_counter()
        self._sync_all()
        t2 = time.perf_counter()
        ph["pack_s"], ph["transfer_s"] = t1 - t0, t2 - t1
        old_verifiers = {n: st.verifier for n, st in self.stages.items()}
        old_ranges = {n: tuple(st.layer_range) for n, st in self.stages.items()}
        # layer modules this rank already holds (a restored node's layers are rebuilt from the
        # snapshot's values, so its modules are re-used too: only the values are untrusted)
        reuse: Dict[int, nn.Module] = {}
        for st in self.stages.values():
            st.remove_hooks()
            a, _ = st.layer_range
            for k, m in enumerate(st.module):
                reuse[a + k] = m
        self.plan = new_plan
        self.stages = {}
        self._build(layer_modules=reuse)
        del reuse
        bt = self._build_times
        ph["rebuild_s"] = bt["materialize_s"] + bt["flatten_s"]
        ph["groups_s"] = bt["groups_s"]
        t3 = time.perf_counter()
        for node, st in self.stages.items():
            a, b = st.layer_range
            for li in range(a, b):
                self._unpack_into(st, li, packed[li])
            st.flat.step_count = step_count
            if st.flat.data is not st.flat.master:
                st.flat.data.copy_(st.flat.master)
            # detector baselines describe the layers a stage held: carry them over only when the
            # stage kept exactly its layers (a stage that took over layers starts a fresh warm-up)
            ov = old_verifiers.get(node)
            if ov is not None and old_ranges.get(node) == tuple(st.layer_range) and ov.S == st.verifier.S:
                st.verifier.adopt(ov)
                st.verifier.rewarm()   # the re-sharded pipeline's dynamics shift: re-warm, gated
        del packed
        self._sync_all()
        ph["unpack_s"] = time.perf_counter() - t3
        self._shape_cache = {}
        self._gsk_cache = {}
        self.refresh_shadows()               # the snapshot ring follows the plan: a fresh committed copy now
        ph["transfer_bytes"] = xfer_bytes
        ph["local_bytes"] = sum(self._packed_numel(li) * 4 for li in range(self.num_layers)
                                if not self.distributed or self.plan.owner_of_layer(li) == self.rank)
        ph["flattened_params"] = bt["flattened_params"]
        ph["materialized_params"] = bt["materialized_params"]
        ph["stages"] = bt["stages"]
        self._migrate_phases = ph
        self._reshard_samples = getattr(self, "_reshard_samples", []) + [ph]
        return moved

    # ================================================================== trusted shadow snapshots
    # SURVEY 5 ("shadow copies of each stage's weights on a neighbour GPU"): when the stages are
    # (re)built and every ``shadow_interval`` steps each stage packs its layers (fp32 master + AdamW
    # moments + buffers, the migration format) and sends them over xGMI to the next
    # ``shadow_copies`` stages of the ring, which keep the copies in HBM (~0.5 GB per GPT-2-medium
    # stage).  The owner's checksum of the packed vector is recorded on every rank.  A periodic
    # copy is committed only when that step's report shows the stage unflagged (the build-time
    # copy at once: the weights come from initialisation, a checkpoint or trusted sources).  A
    # stage later marked compromised is rebuilt from a committed copy held by a trusted holder
    # whose bytes still match the owner's checksum — never from its own (possibly tampered)
    # memory; with no such copy its layers restart from their initial weights.  Metadata (step,
    # layer range, holders, owner checksum) is identical on every rank; only holders keep data.
    def _reset_shadows(self):
        # owner -> committed (step, layer range, primary holder, holders)
        self._shadow_meta: Dict[int, Tuple[int, Tuple[int, int], int, List[int]]] = {}
        self._shadow_pend_meta: Dict[int, Tuple[int, Tuple[int, int], int, List[int]]] = {}
        self._shadow_data: Dict[int, torch.Tensor] = {}      # owner -> committed vector (holders only)
        self._shadow_pend: Dict[int, Tuple[int, torch.Tensor]] = {}
        self._shadow_hash: Dict[int, torch.Tensor] = {}      # owner -> committed owner checksum (every rank)
        self._shadow_pend_hash: Dict[int, torch.Tensor] = {}

    def _shadow_enabled(self) -> bool:
        return self.cfg.shadow_interval > 0 and self.dp == 1 and self.plan.num_stages > 1

    def _shadow_holders(self, node: int) -> List[int]:
        ranks = self.plan.ranks
        i = ranks.index(node)
        k = max(1, min(int(self.cfg.shadow_copies), len(ranks) - 1))
        return [ranks[(i + d) % len(ranks)] for d in range(1, k + 1)]

    def _shadow_holder(self, node: int) -> int:
        return self._shadow_holders(node)[0]

    def _shadow_usable(self, c: int, bad: Sequence[int] = ()) -> bool:
        return self._shadow_source(c, bad) is not None

    def _shadow_source(self, c: int, bad: Sequence[int] = (), verified: Optional[Dict] = None) -> Optional[int]:
        """The holder that serves owner ``c``'s committed copy: the first of its holders that is
        not excluded, not among ``bad`` (the nodes being compromised now), may take tasks and (when
        ``verified`` is given) whose copy still matches the owner's checksum."""
        meta = self._shadow_meta.get(c)
        if meta is None:
            return None
        for h in meta[3]:
            if h in self.excluded or h in bad or not self.trust.can_assign_task(h):
                continue
            if verified is not None and not verified.get((c, h), False):
                continue
            return h
        return None

    def _verify_shadows(self) -> Dict[Tuple[int, int], bool]:
        """(owner, holder) -> the holder's committed copy matches the owner's checksum.  Each rank
        checks the copies it holds; distributed: one all-gather so every rank decides alike."""
        N = self.num_nodes
        mine = torch.zeros(N, dtype=torch.float32, device=self.device)
        for c, vec in self._shadow_data.items():
            ref = self._shadow_hash.get(c)
            if ref is not None:
                ok = torch.equal(dstats.checksum(vec).to(ref.device), ref)
                mine[c] = 1.0 if ok else 0.0
        out: Dict[Tuple[int, int], bool] = {}
        if self.distributed:
            V = all_gather_rows(mine, self.world)
            note_host_sync()
            V = V.cpu()
            for c, meta in self._shadow_meta.items():
                for h in meta[3]:
                    out[(c, h)] = bool(V[h, c] > 0)
        else:
            for c, meta in self._shadow_meta.items():
                for h in meta[3]:
                    out[(c, h)] = bool(mine[c] > 0)
        return out

    def _shadow_slice(self, li: int) -> torch.Tensor:
        for c, meta in self._shadow_meta.items():
            a, b = meta[1]
            if a <= li < b:
                off = sum(self._packed_numel(k) for k in range(a, li))
                return self._shadow_data[c][off:off + self._packed_numel(li)]
        raise KeyError(li)

    @torch.no_grad()
    def _take_shadow(self):
        step = self.global_step
        owners = list(self.plan.ranks)
        for node, rng in zip(self.plan.ranks, self.plan.ranges):
            hs = self._shadow_holders(node)
            self._shadow_pend_meta[node] = (step, tuple(rng), hs[0], hs)
        if self.distributed:
            st = self.my_stage()
            vec = (torch.cat([self._pack_layer(st, li) for li in range(*st.layer_range)]) if st is not None
                   else torch.zeros(0, device=self.device))
            h = dstats.checksum(vec) if st is not None else torch.zeros(3, dtype=torch.float64, device=self.device)
            H = all_gather_rows(h, self.world)
            for node in owners:
                self._shadow_pend_hash[node] = H[node].clone()
            if st is None:
                return
            sends = [(vec, hd) for hd in self._shadow_holders(self.rank)]
            recvs = []
            for o in owners:
                if o != self.rank and self.rank in self._shadow_holders(o):
                    a, b = self.plan.ranges[owners.index(o)]
                    buf = torch.empty(sum(self._packed_numel(li) for li in range(a, b)), dtype=torch.float32,
                                      device=self.device)
                    recvs.append((buf, o))
                    self._shadow_pend[o] = (step, buf)
            self._note_peers(sends, recvs)
            batched_transfer(sends, recvs, meter=self.link_meter)
        else:
            for node, st in self.stages.items():
                dev = self.stages[self._shadow_holder(node)].device
                vec = torch.cat([self._pack_layer(st, li) for li in range(*st.layer_range)])
                self._shadow_pend_hash[node] = dstats.checksum(vec)
                self._shadow_pend[node] = (step, vec.to(dev, copy=True))

    def refresh_shadows(self):
        """Take and commit a snapshot now (stages freshly built from trusted weights: at start-up,
        after a re-shard, after a checkpoint load), so a committed copy exists from step 0 on."""
        if not self._shadow_enabled():
            return
        self._reset_shadows()
        self._take_shadow()
        for owner in list(self._shadow_pend_meta):
            self._commit_one(owner, self.global_step)

    def _commit_one(self, owner: int, step: int) -> None:
        meta = self._shadow_pend_meta.pop(owner)
        data = self._shadow_pend.pop(owner, None)
        if data is not None and data[0] != step:   # a newer snapshot replaced it: keep that one
            self._shadow_pend[owner] = data
            data = None
        self._shadow_meta[owner] = meta
        if owner in self._shadow_pend_hash:
            self._shadow_hash[owner] = self._shadow_pend_hash.pop(owner)
        if data is not None:
            self._shadow_data[owner] = data[1]

    def _commit_shadows(self, step: int, blamed: Sequence[bool], statuses: Sequence[int]):
        bad = (STATUS_CODES[NodeStatus.COMPROMISED], STATUS_CODES[NodeStatus.SUSPICIOUS])
        for owner, meta in list(self._shadow_pend_meta.items()):
            if meta[0] != step:
                continue
            if blamed[owner] or statuses[owner] in bad:
                self._shadow_pend_meta.pop(owner)
                data = self._shadow_pend.pop(owner, None)
                if data is not None and data[0] != step:
                    self._shadow_pend[owner] = data
                self._shadow_pend_hash.pop(owner, None)
                continue
            self._commit_one(owner, step)

    # ================================================================== evaluation
    @torch.no_grad()
    def eval_step(self, batch: Dict[str, torch.Tensor]) -> float:
        """Forward-only loss over the global batch (no detector side effects: reference A21 fixed)."""
        bump_weight_generation()
        M = self.cfg.micro_batches
        inp, tgt = batch["input"], batch["target"]
        if self.dp > 1:
            inp, tgt = inp.chunk(self.dp, 0)[self.replica], tgt.chunk(self.dp, 0)[self.replica]
        inputs, targets = split_micro(inp, M), split_micro(tgt, M)
        total = torch.zeros((), dtype=torch.float32, device=self.device)
        if not self.distributed:
            for i in range(M):
                x = inputs[i]
                for k, node in enumerate(self.plan.ranks):
                    st = self.stages[node]
                    x = self._stage_input(x, st) if k == 0 else x.to(st.device)
                    x, _ = st.forward(x, targets[i].to(st.device) if st.computes_loss else None)
                total += x.float().to(self.device) / M
            return float(total)
        st = self.my_stage()
        if st is not None:
            in_shape, out_shape = self._boundary_shapes(st, inputs[0])
            for i in range(M):
                if st.stage_id == 0:
                    x = self._stage_input(inputs[i], st)
                else:
                    x, _ = self.comm.exchange(recv_prev=(in_shape, self.dtype))
                y, _ = st.forward(x, targets[i].to(st.device) if st.computes_loss else None)
                if st.computes_loss:
                    total += y.float() / M
                else:
                    self.comm.exchange(send_next=y)
        dist.all_reduce(total)
        return float(total) / self.dp

    # ================================================================== checkpoint state
    def stage_state_dicts(self) -> Dict[int, Dict[str, torch.Tensor]]:
        """model_partitions[node] = stage-local state dict (fp32 master weights + buffers)."""
        out = {}
        for node, st in self.stages.items():
            sd = {}
            for i, n in enumerate(st.flat.names):
                sd[n] = st.flat.view(st.flat.master, i).detach().cpu().clone()
            for n, b in st.module.named_buffers():
                sd[n] = b.detach().cpu().clone()
            out[node] = sd
        return out

    def optimizer_state_dicts(self) -> Dict[int, Dict]:
        return {node: st.flat.state_dict() for node, st in self.stages.items()}

    def verifier_state_dicts(self) -> Dict[int, Dict]:
        return {node: st.verifier.state_dict() for node, st in self.stages.items()}

    def trust_state(self) -> Dict[str, torch.Tensor]:
        return {"values": self.t_values.cpu(), "counts": self.t_counts.cpu(), "status": self.t_status.cpu()}

    def load_trust_state(self, sd, partial: bool = False):
        """``partial``: the saved job had a different node count; the first ``len`` entries are
        restored, the rest keep their initial values."""
        for dst, key in ((self.t_values, "values"), (self.t_counts, "counts"), (self.t_status, "status")):
            src = sd[key]
            if partial:
                k = min(dst.numel(), src.numel())
                dst[:k].copy_(src[:k])
            else:
                dst.copy_(src)

    def load_layer_states(self, layers: Dict[int, Dict], step: int):
        """Fill the local stages layer by layer (fp32 master + AdamW moments + buffers) from a saved
        job whose plan differs from this one (utils/checkpoint.load_checkpoint).  Tied parameters
        that the saved stage stored under another layer of their tie group are found there."""
        alias: Dict[Tuple[int, str], List[Tuple[int, str]]] = {}
        for grp in self.ties:
            for m in grp:
                alias[m] = [o for o in grp if o != m]

        def find(kind, li, attr):
            ent = layers.get(li, {}).get(kind, {})
            if attr in ent:
                return ent[attr]
            for lj, aj in alias.get((li, attr), []):
                ent = layers.get(lj, {}).get(kind, {})
                if aj in ent:
                    return ent[aj]
            raise KeyError(f"checkpoint holds no {kind[:-1]} '{attr}' of layer {li}")

        self.t_taint.zero_()      # weights replaced from a checkpoint
        for node, st in self.stages.items():
            a, _ = st.layer_range
            for i, name in enumerate(st.flat.names):
                k, attr = name.split(".", 1)
                m, ea, eas = find("params", a + int(k), attr)
                st.flat.view(st.flat.master, i).copy_(m)
                st.flat.view(st.flat.exp_avg, i).copy_(ea)
                st.flat.view(st.flat.exp_avg_sq, i).copy_(eas)
            for name, b in st.module.named_buffers():
                k, attr = name.split(".", 1)
                b.copy_(find("buffers", a + int(k), attr))
            st.flat.step_count = int(step)
            if st.flat.data is not st.flat.master:
                st.flat.data.copy_(st.flat.master)
            st.param_checksum = None
        bump_weight_generation()
        self.refresh_shadows()    # the loaded weights are the new trusted copy

    def load_stage_states(self, model_sd: Dict[int, Dict], optim_sd: Dict[int, Dict],
                          verifier_sd: Optional[Dict[int, Dict]] = None):
        self.t_taint.zero_()      # weights replaced from a checkpoint
        missing = [n for n in self.stages if n not in optim_sd and n not in model_sd]
        if missing:
            raise KeyError(f"checkpoint holds no state for local stage node(s) {missing}")
        for node, st in self.stages.items():
            if node in optim_sd:
                st.flat.load_state_dict(optim_sd[node])
            elif node in model_sd:
                for i, n in enumerate(st.flat.names):
                    if n in model_sd[node]:
                        st.flat.view(st.flat.master, i).copy_(model_sd[node][n])
                if st.flat.data is not st.flat.master:
                    st.flat.data.copy_(st.flat.master)
            if node in model_sd:
                for n, b in st.module.named_buffers():
                    if n in model_sd[node]:
                        b.copy_(model_sd[node][n])
            if verifier_sd and node in verifier_sd:
                st.verifier.load_state_dict(verifier_sd[node])
            st.param_checksum = None  # weights legitimately replaced
        self.refresh_shadows()        # the loaded weights are the new trusted copy
