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
import os
import time
from collections import deque
from typing import Any, Dict, List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from ..core.trust_manager import STATUS_CODES, TrustManager
from ..ops import stats as dstats
from ..ops.layers import bump_weight_generation
from ..runtime import progress
from ..runtime.commcheck import note_host_sync
from ..runtime.tracing import PhaseTracer
from ..security import stage_verifier as SV
from .attribution import AttributionMixin
from .audit import AuditMixin
from .audit_dist import DistAuditMixin
from .comm import LinkMeter, P2PComm, all_gather_rows
from .commitments import CommitmentMixin
from .dp import DataParallelMixin
from .engine_config import EngineConfig, _resolve_dtype, split_micro  # noqa: F401  (re-exported)
from .partition import make_plan
from .reshard import ReshardMixin, no_gc
from .schedule import ScheduleMixin
from .shadows import ShadowMixin
from .stage import Stage, tied_groups
from .state_io import StateIOMixin

logger = logging.getLogger(__name__)


class PipelineEngine(ScheduleMixin, CommitmentMixin, AuditMixin, DistAuditMixin, AttributionMixin,
                     DataParallelMixin, ReshardMixin, ShadowMixin, StateIOMixin):
    """The engine: construction, communicators, the step (``train_step`` -> schedule ->
    ``_finish_step``), tied-weight all-reduce and evaluation.  Schedules, commitments, audit,
    attribution, data parallelism, re-sharding, shadows and checkpoint state live in the mixin
    modules next to this one."""
    def __init__(self, model: nn.Module, cfg: EngineConfig, trust_manager: Optional[TrustManager] = None,
                 attacker=None, metrics=None, detector=None):
        self.cfg = cfg
        self.model = model                       # CPU master copy: layer skeletons for (re)sharding
        self._init_runtime_state()
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
        if attacker is not None and hasattr(attacker, "public_sketch_fn"):
            attacker.public_sketch_fn = self._public_sketch_of   # public job data (adaptive adversary)
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
        with no_gc():   # the build's timings calibrate the re-shard estimate: no GC pause inside
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

    def _init_runtime_state(self):
        """Every per-engine attribute the mixins use, created here (none lazily)."""
        # communicators (_build_comm): cached process groups, P2P peers per communicator kind
        self._group_cache: Dict[Tuple[str, Tuple[int, ...]], object] = {}
        self._p2p_peers: Dict[str, set] = {}
        self._dir_groups = None                  # async P2P: (activation group, gradient group)
        self._audit_pg = None                    # the audit's weight-shipment communicator
        self._tie_work = None                    # early tied all-reduce in flight
        self._hi_stream = None                   # TDL_COMPUTE_PRIORITY=high stream
        self._built_once = False
        self._build_times: Dict[str, float] = {}
        self._init_build_times: Dict[str, float] = {}
        # per-step schedule / audit state (reset by _train_step)
        self._truth_now: Dict[int, bool] = {}
        self._audit_now = False
        self._audit_ms: List[int] = []           # local mode: the step's audited micro-batches
        self._audit_batch: List[torch.Tensor] = []
        self._audit_targets: List[torch.Tensor] = []
        self._audit_rec: Dict[int, Dict[int, Dict[str, Any]]] = {}
        self._audit_inputs: Dict[int, torch.Tensor] = {}
        self._audit_sent_dx: Dict[int, torch.Tensor] = {}
        self._audit_recv_dy: Dict[int, torch.Tensor] = {}
        self._audit_outputs: Dict[int, torch.Tensor] = {}
        self._early_ship = None                  # (P2P works, mirrors) of the early weight shipment
        self._audit_rng = None                   # distributed auditor's private RNG (audit_dist.py)
        self._audit_cost = {"steps": 0, "host_s": 0.0, "bytes": 0, "sent": 0, "events": [], "seeds": 0,
                            "seed_bytes": 0}
        self._target_log: List[Tuple[int, int, int]] = []
        self._mirrors: Dict[Tuple[int, Tuple[int, int]], Stage] = {}
        # gradient commitments (commitments.py) and optimizer mirrors (audit.py)
        self._gsk_on = False
        self._gsk_run: Dict[int, torch.Tensor] = {}      # public running sketches (targeting)
        self._gring: Dict[int, torch.Tensor] = {}        # [M, n] per-micro-batch contributions
        self._gprev: Dict[int, torch.Tensor] = {}        # [n] running gradient before the next one
        self._gcom: Dict[int, torch.Tensor] = {}         # [M + 2, 8] roots: contributions, applied, master
        self._audit_side: Dict[str, object] = {}         # per device: stream of the mirrors' weight roots
        self._gring_cache: Dict[tuple, Tuple[torch.Tensor, torch.Tensor]] = {}
        self._mirror_epoch = 0                           # bumped on every rank when mirrors go stale
        self._mirror_pending: List = []                  # (mirror, verified gradient, node) to apply
        self._mirror_applied: Dict[int, object] = {}     # node -> its mirror advanced this step (local heal)
        self._seed_mark = None                           # (plan, range, epoch) my auditor's mirror was seeded for
        self._tkey_trash: List[str] = []                 # store keys of last step's tie-key parts (audit_dist.py)
        self._gsk_cache: Dict[tuple, object] = {}
        # attribution (attribution.py)
        self._proof: Optional[torch.Tensor] = None
        self._proof_kind: Optional[torch.Tensor] = None
        self._orders_key = None
        self._orders: List[torch.Tensor] = []
        # caches
        self._shape_cache: Dict[tuple, tuple] = {}
        self._idx_cache: Dict[tuple, torch.Tensor] = {}
        # data parallelism (dp.py)
        self._dp_sidx: Optional[torch.Tensor] = None
        self._dp_excluded: Optional[torch.Tensor] = None
        self._dp_cos: Optional[torch.Tensor] = None
        # re-sharding (reshard.py)
        self._reshard_samples: List[Dict[str, float]] = []
        self._migrate_phases: Dict[str, float] = {}
        self._old_owner: Dict[int, int] = {}
        self._checkpoints: List[Tuple[str, int]] = []   # (path, step) saved / loaded (re-shard source)

    def _public_sketch_of(self, node: int):
        """(public GradSketch, this step's window offset) of a local stage: everything about it
        derives from the job seed, the step and the layer range (what an adaptive adversary knows)."""
        st = self.stages.get(node)
        if st is None:
            return None, 0
        sk = self._sketch_for(st)
        return sk, sk.offset(self.cfg.seed, self.global_step)

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
        vk.setdefault("early_gate", self._built_once)
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
        # the split-K reduce of the last micro-batch's weight gradients may complete main_grad on
        # the verifier's side stream (stage.py _arm_sinks) only where nothing else reads the
        # gradient before the step tail joins that stream: no commitments / audit, no replicas, no
        # gradient attacker
        side_ok = (not (self.cfg.audit and self.plan.num_stages > 1) and self.dp == 1 and self.attacker is None)
        for st in self.stages.values():
            st.set_early_stats(tied)
            st.side_reduce_ok = side_ok
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
        if not self.distributed:
            return
        s = self.plan.stage_of_rank(self.rank)
        prev = self.plan.ranks[s - 1] if s is not None and s > 0 else None
        nxt = self.plan.ranks[s + 1] if s is not None and s + 1 < self.plan.num_stages else None
        self.comm = P2PComm(prev, nxt, self.device)
        for peer in (prev, nxt):
            if peer is not None:
                self._p2p_peers.setdefault("default" if self.p2p_mode != "async" else "dir", set()).add(peer)
        if self.p2p_mode == "async" and self._dir_groups is None:
            # one communicator for activations (stage s -> s+1), one for activation gradients
            # (s+1 -> s): each carries one-way, in-order traffic per neighbour pair
            everyone = list(range(self.world))
            self._dir_groups = (self._group("act", everyone), self._group("grad", everyone))
        if self.cfg.audit and self._audit_pg is None:
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
        self._p2p_peers.setdefault(kind, set()).update(int(p) for _, p in list(sends) + list(recvs))

    def comm_inventory(self) -> Dict[str, object]:
        """Per-rank communicator / stream count by purpose, against the HIP hardware-queue budget.
        Communicators: the default group's, one per cached group this rank belongs to, and one
        2-rank P2P communicator per (group, peer) this rank has exchanged with."""
        groups = [{"purpose": p, "members": list(m)} for (p, m) in self._group_cache]
        mine = [g for g in groups if self.rank in g["members"]]
        p2p = {k: sorted(v) for k, v in self._p2p_peers.items()}
        n_p2p = sum(len(v) * (2 if k == "dir" else 1) for k, v in p2p.items())
        n_comms = (1 if self.distributed else 0) + len(mine) + n_p2p
        from ..ops.side_stream import WgradSide
        # compute + verification side streams + weight-gradient side streams + RCCL streams
        streams = 1 + len(self.stages) + WgradSide.count() + len(self._audit_side) + n_comms
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
        s = self._hi_stream
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
        # local mode: the audited micro-batches (k of M, the monitored one among them) are drawn from
        # the engine's private RNG now; distributed auditors draw theirs after the step (audit_dist.py)
        self._audit_ms = []
        if self._audit_now and not self.distributed and self._mon_idx >= 0:
            k = max(1, min(int(self.cfg.audit_micro_k), M))
            rest = [m for m in range(M) if m != self._mon_idx]
            self._audit_ms = [self._mon_idx] + self._mon_rng.sample(rest, k - 1)
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

    def begin_step(self) -> int:
        """Open an optimizer step (``train_step`` does this itself; the reference per-phase API —
        DistributedTrainer.forward_pass / backward_pass / optimizer_step — calls it explicitly)."""
        self._consume_reports(upto=self.global_step + 1 - self.REPORT_LAG)
        if self.device.type == "cuda":
            from ..ops.side_stream import WgradSide
            WgradSide.join_all()
        bump_weight_generation()   # weights may have changed since the last step (update, re-shard, restore, load)
        self._gsk_on = False       # the per-phase API (external backward) commits no gradient sketches
        self._truth_now = {}
        self.global_step += 1
        self.trust.advance_step(self.global_step)
        return self.global_step

    def end_step(self, loss: Optional[torch.Tensor], truth: Optional[Dict[int, bool]] = None) -> Optional[float]:
        """Close a step whose gradients are already accumulated in the stages' flat buffers (by an
        external ``loss.backward()``): tied all-reduce, verification digest, attribution, trust
        update, global-norm clipping + quarantine, fused AdamW — the same tail as ``train_step``.
        No gradient commitments are taken on this path, so the auditors' mirrors go stale."""
        self._invalidate_mirrors()
        self._mirror_pending = []
        self._finish_step(None if loss is None else loss.detach(), dict(truth or {}))
        self.tracer.end_step(self.global_step)
        self.tracer.resolve()
        return self.last_loss



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
        if self._tie_work is not None or not self.tie_members or self.rank not in self.tie_members:
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
        work = self._tie_work
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
        cache = self._idx_cache
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
            # weight-shipping mode (no mirror): the root of the weights in use this step (= after the
            # last update); the auditor hashes the weights it receives and every rank compares
            if self.distributed and self._audit_now and not self._gsk_on:
                from ..security.grad_audit import hash_row
                d[SV.D_WHASH:SV.D_WHASH + 8].copy_(hash_row(self._tensor_root(st.flat.data)))
            else:
                d[SV.D_WHASH:SV.D_WHASH + 8].fill_(-1.0)
            if self.cfg.param_integrity:
                d[SV.D_PARAM_FLAG:SV.D_PARAM_FLAG + 1].copy_(self._integrity_flag(st))
                if self.attacker is not None and getattr(self.attacker, "lies_about_integrity", None) \
                        and self.attacker.lies_about_integrity(node, self.global_step):
                    d[SV.D_PARAM_FLAG:SV.D_PARAM_FLAG + 1].fill_(0.0)   # a rank lying about its own check
            self._write_commitments(node, st, d)
            rows.append((node, d))
        if self._audit_now or self._gsk_on:
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
        if self._gsk_on:
            # mirror mode: the skip decision comes from the digest alone (its auditor's mirror takes
            # the same one: audit.py _skip_decision)
            for node, st in self.stages.items():
                st.verifier.ctrl[1:2].copy_(self._skip_decision(D, evidence, node).to(st.device))
        elif self.quarantine_on_evidence:
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
            sq = self._clip_sumsq_audited(D) if self._gsk_on else D[:, SV.D_GRAD_SUMSQ]
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
        if self._mirror_pending:
            # before the stages' own updates: in local mode a mirror reads its stage's gradient buffer
            self._mirror_update(D, evidence, total_sumsq)
        for node, st in self.stages.items():
            st.verifier.set_clip_scale(total_sumsq.to(st.device), self.cfg.adamw.max_grad_norm)
            cur = st._cur_checksum
            if self.cfg.param_integrity and cur is not None:
                # the weights must still be those checksummed at the start of the step
                st._tail_flag = (dstats.checksum(st.flat.data) != cur).any().float().reshape(1)
            st.flat.adamw_step(self.cfg.adamw, ctrl=st.verifier.ctrl)
            if self._gsk_on and not self.distributed:
                self._heal_from_mirror(node, st)
            if self.cfg.param_integrity:
                st.param_checksum = dstats.checksum(st.flat.data, st.param_checksum)
        self.tracer.end(to)
        if self._shadow_enabled() and self.global_step % self.cfg.shadow_interval == 0:
            self._take_shadow()
        if self.dp > 1 and self.cfg.param_audit_interval and self.global_step % self.cfg.param_audit_interval == 0:
            self._audit_params()
        # queue the host report (pinned, non-blocking)
        if self._audit_now or self._gsk_on:
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
        self._pending.append((self.global_step, self.epoch, host, ev, dict(truth), list(self.last_ranks()),
                              (self.plan.version, bool(self._gsk_on))))

    def close(self):
        if self.heartbeat is not None:
            self.heartbeat.stop()
            self.heartbeat = None



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
