"""Task reassignment (re-sharding) of ``PipelineEngine``: exclude compromised stages, re-plan the
layers over the trusted ranks and migrate fp32 master + AdamW state (over xGMI when distributed),
with a measured migration-time model.  Reference: reassign_node_tasks / estimate_migration_time /
perform_task_reassignment (distributed_trainer.py:324-380), a no-op there.
"""
from __future__ import annotations

import gc
import logging
import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from ..runtime.commcheck import note_host_sync
from .comm import batched_transfer, broadcast_ints
from .partition import PlacementPlan, make_plan
from .stage import Stage

logger = logging.getLogger(__name__)


class no_gc:
    """Automatic Python garbage collection off for a block (re-enabled on exit if it was on).  A
    generation-2 collection over the engine's module graph costs 70-145 ms; landing inside a
    re-shard it tripled the measured rebuild and skewed the calibration (r5_cfg_full2.jsonl
    ``rebuild_gc_s``).  The collection then runs at a later allocation instead."""

    def __enter__(self):
        self.was = gc.isenabled()
        gc.disable()
        return self

    def __exit__(self, *exc):
        if self.was:
            gc.enable()
        return False


class _RebuildProbe:
    """Diagnostics of a stage rebuild: seconds spent in Python garbage collections that ran inside
    it and the device memory the caching allocator had to newly reserve (hipMalloc) for it — the
    two suspects behind rebuilds 2-3x slower than the median (profiles/r5_cfg_full.jsonl)."""

    def __init__(self, device: torch.device):
        self.device = device
        self.gc_s = 0.0
        self._t = 0.0

    def _cb(self, phase, info):
        if phase == "start":
            self._t = time.perf_counter()
        else:
            self.gc_s += time.perf_counter() - self._t

    def __enter__(self):
        self.res0 = torch.cuda.memory_reserved(self.device) if self.device.type == "cuda" else 0
        gc.callbacks.append(self._cb)
        return self

    def __exit__(self, *exc):
        gc.callbacks.remove(self._cb)
        res1 = torch.cuda.memory_reserved(self.device) if self.device.type == "cuda" else 0
        self.new_reserved = max(0, res1 - self.res0)
        return False


class ReshardMixin:
    """Re-sharding (mixed into ``PipelineEngine``)."""

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
        groups: communicator set-up of the new plan (cached groups cost nothing);
        other: what a re-shard spends outside those phases (device syncs, the fresh shadow ring),
        measured as wall minus phases.
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
               + cal["groups_s"] + cal["other_s"])
        return est

    def _reshard_calibration(self) -> Dict[str, float]:
        """Rates behind ``estimate_migration_time``: the median over this engine's initial build and
        every re-shard measured so far (``_reshard_samples``; a median keeps one slow outlier, e.g.
        an allocator flush during a rebuild, from skewing the next prediction)."""
        bt = self._init_build_times or self._build_times
        mat_rate = bt.get("materialize_s", 0.0) / max(1, bt.get("materialized_params", 1))
        flat = [bt.get("flatten_s", 0.0) / max(1, bt.get("flattened_params", 1))]
        # priors (MI355X, measured on GPT-2-medium re-shards, profiles/r5_cfg_calib.jsonl): pack +
        # unpack gather / scatter per-layer slices at ~300 GB/s, not a bulk copy's rate; ~6 ms of
        # syncs and shadow refresh outside the timed phases
        gpu = self.device.type == "cuda"
        copy = [1.0 / (300e9 if gpu else 4e9)]
        groups = [0.0]
        other = [0.006 if gpu else 0.0]
        for ph in self._reshard_samples:
            if ph.get("local_bytes"):
                copy.append((ph["pack_s"] + ph["unpack_s"]) / ph["local_bytes"])
            if ph.get("flattened_params"):
                flat.append(max(0.0, ph["rebuild_s"] - ph["materialized_params"] * mat_rate) / ph["flattened_params"])
            groups.append(ph.get("groups_s", 0.0))
            if "other_s" in ph:
                other.append(ph["other_s"])

        def med(v):   # true median (an even count averages the middle two: the upper one alone let
            #           one slow first re-shard set the next prediction, r5_cfg_full.jsonl config 5 s1)
            v = sorted(v)
            n = len(v)
            return v[n // 2] if n % 2 else 0.5 * (v[n // 2 - 1] + v[n // 2])
        return {"copy_s_per_byte": med(copy), "flatten_s_per_param": med(flat),
                "materialize_s_per_param": mat_rate, "groups_s": med(groups), "other_s": med(other)}

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
        # a trusted holder whose copy verifies; when that shadow is missing or older than
        # 2 x shadow_interval, from the newest checkpoint saved before the node's first blame (if it
        # is newer than the shadow); else from the initial weights
        now = step if step is not None else self.global_step
        verified = self._verify_shadows() if self._shadow_meta else {}
        sources = {c: self._shadow_source(c, compromised, verified) for c in compromised}
        from_ckpt: Dict[int, Tuple[str, int]] = {}
        stale: List[int] = []
        for c in compromised:
            sstep = self._shadow_meta[c][0] if sources[c] is not None else None
            if sstep is None or (self.cfg.shadow_interval > 0 and now - sstep > 2 * self.cfg.shadow_interval):
                stale.append(c)
                ck = self._checkpoint_before_blame(c)
                if ck is not None and (sstep is None or ck[1] > sstep):
                    from_ckpt[c] = ck
                    sources[c] = None
        restored = {c: self._shadow_meta[c][0] for c in compromised if sources[c] is not None}
        fresh = [c for c in compromised if sources[c] is None and c not in from_ckpt]
        if stale:
            logger.warning("stale or missing shadow for %s (step %d, interval %d): %s", stale, now,
                           self.cfg.shadow_interval, {c: from_ckpt.get(c, ("shadow" if c in restored else "initial",))[-1]
                                                      for c in stale})
        if fresh:
            logger.warning("no verified shadow or checkpoint for %s: their layers restart from the initial weights", fresh)
        to_move = sum(self._layer_numel(li) for li in range(self.num_layers)
                      if self.plan.owner_of_layer(li) != new_plan.owner_of_layer(li) or
                      any(self.plan.owner_of_layer(li) == c for c in compromised))
        predicted = self.estimate_migration_time(to_move, plan=new_plan)   # before the move: a prediction
        t0 = time.perf_counter()
        with no_gc():
            moved = self._migrate(new_plan, restore={c: sources[c] for c in restored}, fresh=fresh, ckpt=from_ckpt)
        dt = time.perf_counter() - t0
        ph = self._migrate_phases
        ph["other_s"] = max(0.0, dt - sum(ph.get(k, 0.0) for k in ("pack_s", "transfer_s", "rebuild_s", "groups_s",
                                                                   "unpack_s")))
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
               "restored_from_checkpoint": {c: ck[1] for c, ck in from_ckpt.items()},
               "restored_from_initial": fresh,
               "stale_shadow": stale,
               "shadow_holders": {c: sources[c] for c in restored},
               "plan": new_plan.describe()}
        self.reassignment_history.append(rec)
        logger.warning("Reassigned tasks from %s -> %s in %.3fs; new plan %s", compromised, to_nodes, dt,
                       new_plan.describe())

    def note_checkpoint(self, path: str, step: int) -> None:
        """A complete checkpoint of the whole job was saved / loaded at ``step`` (utils/checkpoint.py):
        a re-shard source for compromised stages whose shadow is stale."""
        self._checkpoints.append((path, int(step)))
        self._checkpoints = self._checkpoints[-8:]

    def _checkpoint_before_blame(self, c: int) -> Optional[Tuple[str, int]]:
        """The newest noted checkpoint taken before node ``c``'s first blame since its last
        re-shard (its weights then predate every detected tamper of this episode)."""
        since = max([r["step"] for r in self.reassignment_history if "step" in r] + [-1])
        blames = [a["step"] for a in self.attack_history if a.get("node_id") == c and a["step"] > since]
        first = min(blames) if blames else self.global_step
        cands = [(p, st) for p, st in self._checkpoints if st < first]
        seen = torch.tensor([1.0 if os.path.exists(p) else 0.0 for p, _ in cands] or [0.0], device=self.device)
        if self.distributed:
            # every rank must restore from the same source: only a checkpoint visible on ALL ranks
            # counts (a non-shared filesystem would otherwise split the re-shard)
            dist.all_reduce(seen, op=dist.ReduceOp.MIN)
        note_host_sync()
        ok = seen.tolist()
        cands = [c for c, v in zip(cands, ok) if v > 0]
        return max(cands, key=lambda x: x[1]) if cands else None

    def _pack_from_checkpoint(self, layers: Dict[int, Dict], li: int, device) -> torch.Tensor:
        """Layer ``li`` in the migration format from a checkpoint's layer states
        (utils/checkpoint._layer_states; a tied parameter may be stored under another member)."""
        alias: Dict[Tuple[int, str], List[Tuple[int, str]]] = {}
        for grp in self.ties:
            for m in grp:
                alias[m] = [o for o in grp if o != m]

        def find(kind, attr):
            for lj, aj in [(li, attr)] + alias.get((li, attr), []):
                ent = layers.get(lj, {}).get(kind, {})
                if aj in ent:
                    return ent[aj]
            raise KeyError(f"checkpoint holds no {kind[:-1]} '{attr}' of layer {li}")
        parts = []
        for name, _ in self.layers[li].named_parameters(remove_duplicate=False):
            parts += [t.reshape(-1).float() for t in find("params", name)]
        for name, _ in self.layers[li].named_buffers():
            parts.append(find("buffers", name).reshape(-1).float())
        return torch.cat(parts).to(device) if parts else torch.zeros(0, device=device)

    def _ckpt_layers(self, ckpt: Dict[int, Tuple[str, int]], old_plan, want: Sequence[int]) -> Dict[int, Dict]:
        """Layer states of the layers in ``want`` from the checkpoints in ``ckpt`` (node -> (path,
        step)); each layer from the checkpoint of the node that held it."""
        from ..utils.checkpoint import _layer_states
        out: Dict[int, Dict] = {}
        by_path: Dict[str, List[int]] = {}
        for c, (path, _) in ckpt.items():
            a, b = old_plan.ranges[old_plan.ranks.index(c)]
            by_path.setdefault(path, []).extend(li for li in range(a, b) if li in want)
        for path, lis in by_path.items():
            ck = torch.load(path, map_location="cpu", weights_only=True)
            layers, _ = _layer_states(path, ck, PlacementPlan.from_list(ck["plan"]), set(lis))
            # tied parameters: the layer states of the other tie members too
            extra = {lj for grp in self.ties for m in grp for lj, _ in grp if m[0] in lis} - set(layers)
            if extra:
                more, _ = _layer_states(path, ck, PlacementPlan.from_list(ck["plan"]), extra)
                layers.update(more)
            out.update(layers)
        return out

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
                 fresh: Sequence[int] = (), ckpt: Optional[Dict[int, Tuple[str, int]]] = None) -> int:
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
        from_ck = {li for c in (ckpt or {}) for li in range(self.num_layers) if old_plan.owner_of_layer(li) == c}
        ck_layers: Dict[int, Dict] = {}
        if from_ck:
            mine = {li for li in from_ck if not self.distributed or new_plan.owner_of_layer(li) == self.rank}
            ck_layers = self._ckpt_layers(ckpt, old_plan, mine) if mine else {}
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
                if li in from_init or li in from_ck:
                    if dst == self.rank:
                        packed[li] = (self._pack_from_checkpoint(ck_layers, li, self.device) if li in from_ck
                                      else self._pack_initial(li, self.device))
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
                elif li in from_ck:
                    packed[li] = self._pack_from_checkpoint(ck_layers, li, self.stages[src].device)
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
        with _RebuildProbe(self.device) as probe:
            self._build(layer_modules=reuse)
        del reuse
        bt = self._build_times
        ph["rebuild_s"] = bt["materialize_s"] + bt["flatten_s"]
        ph["rebuild_gc_s"] = probe.gc_s
        ph["rebuild_new_reserved_bytes"] = probe.new_reserved
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
        self._gring_cache = {}               # contribution rings of the old layout
        self.refresh_shadows()               # the snapshot ring follows the plan: a fresh committed copy now
        ph["transfer_bytes"] = xfer_bytes
        ph["local_bytes"] = sum(self._packed_numel(li) * 4 for li in range(self.num_layers)
                                if not self.distributed or self.plan.owner_of_layer(li) == self.rank)
        ph["flattened_params"] = bt["flattened_params"]
        ph["materialized_params"] = bt["materialized_params"]
        ph["stages"] = bt["stages"]
        self._migrate_phases = ph
        self._reshard_samples.append(ph)
        return moved
