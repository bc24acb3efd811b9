"""Checkpoint save / load / consolidate in the reference's top-level layout.

Reference (distributed_trainer.py:448-463): ``torch.save`` of
``{epoch, global_step, model_partitions{node: state_dict}, optimizers{node: state},
trust_scores{i: float}, attack_history, reassignment_history}`` to
``checkpoints/checkpoint_step_{N}.pt`` (the directory was never created: A7; there was no load).

Here: the directory is created; local mode writes one file in exactly that layout; distributed mode
writes one shard per rank (``checkpoint_step_{N}.rank{r}.pt``, holding that rank's
``model_partitions`` / ``optimizers`` entries) plus a rank-0 manifest with every other key, and
``consolidate`` merges them back into the single reference dict.  Extra keys restore the full
trust/detection state on resume: ``plan``, ``trust_manager``, ``device_trust``, ``verifiers``,
``detector``, ``config``.  Everything is tensors / plain containers, so ``torch.load(...,
weights_only=True)`` loads it.
"""
from __future__ import annotations

import glob
import json
import logging
import os
from dataclasses import asdict
from typing import Dict, Optional, Sequence, Set, Tuple

import torch
import torch.distributed as dist

from ..runtime.elastic import node_ids_from_env

logger = logging.getLogger(__name__)


def _jsonable(obj):
    return json.loads(json.dumps(obj, default=lambda o: getattr(o, "value", str(o))))


def _base_dict(trainer) -> Dict:
    e = trainer.engine
    return {
        "epoch": trainer.current_epoch,
        "epoch_batch": int(getattr(trainer, "epoch_batch", 0)),  # batches of `epoch` already trained
        "global_step": e.global_step,
        "trust_scores": {i: trainer.trust_manager.get_trust_score(i) for i in range(trainer.config.num_nodes)},
        "attack_history": _jsonable(e.attack_history),
        "reassignment_history": _jsonable(e.reassignment_history),
        "plan": e.plan.to_list(),
        "granularity": getattr(e, "granularity", "block"),
        "trust_manager": _jsonable(trainer.trust_manager.state_dict()),
        "device_trust": e.trust_state(),
        "detector": _jsonable(trainer.attack_detector.state_dict()),
        "config": _jsonable(asdict(trainer.config)),
        # physical identity of each node (its generation-0 rank under the elastic supervisor)
        "node_ids": node_ids_from_env(trainer.config.num_nodes),
        "excluded": [int(n) for n in getattr(e, "excluded", [])],
    }


def _atomic_save(obj, path: str):
    """write-then-rename: a process killed mid-write never leaves a truncated file under `path`"""
    tmp = f"{path}.tmp{os.getpid()}"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_checkpoint(trainer, path: Optional[str] = None) -> str:
    e = trainer.engine
    e.flush()
    ckdir = trainer.config.checkpoint_dir
    if path is None:
        path = os.path.join(ckdir, f"checkpoint_step_{e.global_step}.pt")
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    parts = {"model_partitions": e.stage_state_dicts(), "optimizers": e.optimizer_state_dicts(),
             "verifiers": e.verifier_state_dicts()}
    if not e.distributed:
        ck = _base_dict(trainer)
        ck.update(parts)
        _atomic_save(ck, path)
    else:
        shard = path.replace(".pt", f".rank{e.rank}.pt")
        _atomic_save({"rank": e.rank, **parts}, shard)
        ck = _base_dict(trainer) if e.rank == 0 else None
        # the manifest is written only once every shard is on disk (a rank lost mid-save leaves no
        # manifest, so `latest_checkpoint` falls back to the previous complete checkpoint)
        dist.barrier()
        if e.rank == 0:
            ck["model_partitions"] = {}
            ck["optimizers"] = {}
            ck["shards"] = [os.path.basename(path.replace(".pt", f".rank{r}.pt")) for r in range(e.world)]
            _atomic_save(ck, path)
        dist.barrier()
    e.note_checkpoint(path, e.global_step)
    logger.info("Checkpoint saved: %s", path)
    return path


def _shard_path(path: str, shard: str) -> str:
    sp = os.path.join(os.path.dirname(path), shard)
    if not os.path.exists(sp):
        raise FileNotFoundError(f"checkpoint {path}: shard {shard} is missing (refusing to resume a stage "
                                f"from freshly initialised weights)")
    return sp


def consolidate(path: str, nodes: Optional[Sequence[int]] = None) -> Dict:
    """Merge a sharded checkpoint into the reference's single top-level dict.  ``nodes``: load only
    these ranks' shards (a resuming rank needs its own, not every rank's).  A listed shard that is
    missing raises: silently resuming a stage from fresh weights is worse than failing."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    shards = ck.pop("shards", [])
    for r, shard in enumerate(shards):
        if nodes is not None and r not in nodes:
            continue
        s = torch.load(_shard_path(path, shard), map_location="cpu", weights_only=True)
        for key in ("model_partitions", "optimizers", "verifiers"):
            ck.setdefault(key, {}).update(s.get(key, {}))
    return ck


def _layer_states(path: str, ck: Dict, saved_plan, want: Set[int]) -> Tuple[Dict[int, Dict], int]:
    """Per-layer optimizer state {layer: {"params": {attr: (master, exp_avg, exp_avg_sq)},
    "buffers": {attr: tensor}}} for the layers in ``want``, read from the saved stages that held
    them (stage-local names ``"<i>.<attr>"`` -> global layer ``a + i``); only those stages'
    shards are loaded.  Also returns the saved optimizer step count."""
    shards = ck.get("shards")
    out: Dict[int, Dict] = {}
    step = 0
    for node, (a, b) in zip(saved_plan.ranks, saved_plan.ranges):
        if not any(a <= li < b for li in want):
            continue
        if shards is not None:
            sh = torch.load(_shard_path(path, shards[node]), map_location="cpu", weights_only=True)
            opt, model = sh["optimizers"].get(node), sh["model_partitions"].get(node, {})
        else:
            opt, model = ck["optimizers"].get(node), ck["model_partitions"].get(node, {})
        if opt is None:
            raise KeyError(f"checkpoint {path}: no optimizer state for saved stage on node {node}")
        step = max(step, int(opt["step"]))
        off = 0
        for name, shp in zip(opt["names"], opt["shapes"]):
            n = int(torch.Size(shp).numel())
            i, attr = name.split(".", 1)
            li = a + int(i)
            if li in want:
                ent = out.setdefault(li, {"params": {}, "buffers": {}})
                ent["params"][attr] = tuple(opt[k][off:off + n].view(shp) for k in ("master", "exp_avg", "exp_avg_sq"))
            off += n
        pnames = set(opt["names"])
        for name, t in model.items():
            if name in pnames:
                continue
            i, attr = name.split(".", 1)
            li = a + int(i)
            if li in want:
                out.setdefault(li, {"params": {}, "buffers": {}})["buffers"][attr] = t
    return out, step


def _node_map(saved_ids, live_ids) -> Dict[int, int]:
    """live node index -> saved node index of the same physical node (absent: a node the saved job
    did not have, which starts fresh)."""
    where = {int(p): j for j, p in enumerate(saved_ids)}
    return {i: where[int(p)] for i, p in enumerate(live_ids) if int(p) in where}


def _saved_node_map(ck: Dict, live: int) -> Dict[int, int]:
    """live rank -> saved node index of the same PHYSICAL node (see _resize_trust)."""
    saved_n = int(ck["device_trust"]["values"].numel()) if "device_trust" in ck else \
        int(ck.get("trust_manager", {}).get("num_nodes", live))
    saved_ids = ck.get("node_ids") or list(range(saved_n))
    return _node_map(saved_ids, node_ids_from_env(live))


def resume_plan_ranks(ck: Dict, saved_ranks, live: int, pp: int):
    """Where a saved plan's stages can run in a job of ``live`` ranks.

    The saved plan names SAVED node indices; after an elastic restart on survivors those are
    different ranks (or gone).  Returns ``(translated_ranks or None, excluded_live_ranks)``:
    the saved ranks translated through the physical node ids, or None when a stage's node is gone,
    out of the pipeline, or was excluded as compromised (then the caller re-plans over the live
    ranks minus the excluded ones, so a compromised node never gets a stage back)."""
    m = _saved_node_map(ck, live)
    inv = {j: i for i, j in m.items()}
    saved_ex = {int(n) for n in ck.get("excluded", [])}
    live_ex = sorted(i for i, j in m.items() if j in saved_ex)
    out = [inv.get(int(r)) for r in saved_ranks]
    ok = len(out) <= pp and all(r is not None and r < pp and r not in live_ex for r in out)
    return (out if ok else None), live_ex


def _resize_trust(trainer, ck: Dict, live: int):
    """Trust state of a job resumed on ``live`` nodes.  Node records follow the PHYSICAL node: the
    checkpoint's ``node_ids`` and this job's (TDL_ELASTIC_NODE_IDS) map each live node to the saved
    record of the same node, so losing rank 0 or 1 of 3 does not hand the lost node's trust or
    COMPROMISED status to whichever survivor inherits its index.  Retired nodes' records stay in the
    attack / reassignment histories; nodes the saved job did not have start fresh."""
    tm = trainer.trust_manager
    m = _saved_node_map(ck, live)
    if "trust_manager" in ck:
        tm.load_state_dict(ck["trust_manager"])
        old_scores, old_status, old_metrics = tm.trust_scores, tm.node_status, tm.node_metrics
        old_attacks, old_last = tm.attack_history, tm._last_step
        tm.trust_scores, tm.node_status, tm.node_metrics = {}, {}, {}
        tm.attack_history = type(old_attacks)(list)
        tm._last_step = {}
        tm.num_nodes = 0
        for i in range(live):
            j = m.get(i)
            if j is not None and j in old_scores:
                tm.trust_scores[i] = old_scores[j]
                tm.node_status[i] = old_status[j]
                tm.node_metrics[i] = old_metrics[j]
                if j in old_attacks:
                    tm.attack_history[i] = list(old_attacks[j])
                if j in old_last:
                    tm._last_step[i] = old_last[j]
        tm.num_nodes = live
        for i in range(live):
            if i not in tm.trust_scores:
                tm.initialize_node(i)
    tm.resize(live)
    if "device_trust" in ck:
        sd = ck["device_trust"]
        cur = trainer.engine.trust_state()
        for key in cur:
            for i, j in m.items():
                if j < sd[key].numel() and i < cur[key].numel():
                    cur[key][i] = sd[key][j]
        trainer.engine.load_trust_state(cur)
    # nodes excluded for compromise stay excluded — the same physical nodes, under their new ranks
    saved_ex = {int(n) for n in ck.get("excluded", [])}
    trainer.engine.excluded = sorted(i for i, j in m.items() if j in saved_ex)


def load_checkpoint(trainer, path: str):
    """Restore weights, optimizer state, trust + detector state.

    * same plan as the live engine: each rank reads only its own shard;
    * a different plan that this job can host (e.g. saved after a re-shard): the saved plan is
      adopted and the stages rebuilt;
    * a different world size (a restart with fewer / more ranks, e.g. after ``abort_on_offline``
      took a node out): rank 0 re-plans the saved layers over the live ranks, the plan is
      broadcast (``broadcast_ints``) so every rank builds the same one, and each rank assembles its
      new stages layer by layer from the saved stages that held them (only those shards are read).
    The reference has no load path at all (distributed_trainer.py:448-463 only saves)."""
    from ..parallel.comm import broadcast_ints
    from ..parallel.partition import PlacementPlan, make_plan
    e = trainer.engine
    ck = torch.load(path, map_location="cpu", weights_only=True)
    saved_plan = PlacementPlan.from_list(ck["plan"])
    g = ck.get("granularity", "block")
    if g != getattr(e, "granularity", "block"):
        e.set_granularity(g)  # layer indices of the saved plan refer to that unit size
        e._build()
    dp = getattr(e, "dp", 1)
    # the saved plan's ranks are SAVED node indices: translate them to this job's ranks through the
    # physical node ids first (after a rank shift an excluded node must not get a stage)
    moved, live_ex = resume_plan_ranks(ck, saved_plan.ranks, e.num_nodes, e.pp)
    # with data-parallel replicas the manifest holds replica 0's plan; replicas share its layout
    same = (moved == e.plan.ranks or dp > 1) and saved_plan.ranges == e.plan.ranges
    hostable = moved is not None
    if same:
        # each rank reads its own shard (a DP replica's stage node is its own rank)
        full = consolidate(path, nodes=sorted(e.stages) if e.distributed else None)
        e.load_stage_states(full["model_partitions"], full["optimizers"], full.get("verifiers") or {})
    elif dp > 1:
        raise ValueError("resuming a data-parallel job under a different pipeline layout is not supported")
    else:
        if hostable:
            new_plan = PlacementPlan(list(moved), list(saved_plan.ranges), saved_plan.version)
        else:
            live = [r for r in range(e.pp) if r not in live_ex][: e.num_layers]
            new_plan = make_plan(e.costs, live, saved_plan.version + 1, e.cfg.balanced_partition)
        if e.distributed:
            new_plan = PlacementPlan.from_list(broadcast_ints(new_plan.to_list() if e.rank == 0 else None, 0,
                                                              e.device))
        e.plan = new_plan
        e._build()
        want = {li for st in e.stages.values() for li in range(*st.layer_range)}
        layers, step = _layer_states(path, ck, saved_plan, want)
        e.load_layer_states(layers, step)
        if not hostable:
            e.reassignment_history.append({
                "event": "resume_replan", "from_plan": saved_plan.describe(), "plan": new_plan.describe(),
                "step": int(ck["global_step"]), "from_nodes": [r for r in saved_plan.ranks if r >= e.num_nodes],
                "to_nodes": list(new_plan.ranks)})
    e.global_step = int(ck["global_step"])
    trainer.current_epoch = int(ck["epoch"])
    trainer.epoch_batch = int(ck.get("epoch_batch", 0))
    hist = list(ck.get("reassignment_history", []))
    e.attack_history[:] = list(ck.get("attack_history", []))
    e.reassignment_history[:] = hist + [r for r in e.reassignment_history if r.get("event") == "resume_replan"]
    _resize_trust(trainer, ck, e.num_nodes)
    if "detector" in ck:
        trainer.attack_detector.load_state_dict(ck["detector"])
    trainer.config.num_nodes = e.num_nodes
    e.note_checkpoint(path, e.global_step)
    logger.info("Checkpoint loaded: %s (step %d, plan %s)", path, e.global_step, e.plan.describe())


def is_complete(path: str) -> bool:
    """A manifest whose listed shards all exist (or a local single-file checkpoint)."""
    try:
        ck = torch.load(path, map_location="cpu", weights_only=True)
    except Exception as exc:  # truncated / unreadable
        logger.warning("checkpoint %s unreadable: %s", path, exc)
        return False
    return all(os.path.exists(os.path.join(os.path.dirname(path), sh)) for sh in ck.get("shards", []))


def latest_checkpoint(ckdir: str) -> Optional[str]:
    """Newest COMPLETE checkpoint in ``ckdir`` (every listed shard present), or None."""
    files = [f for f in glob.glob(os.path.join(ckdir, "checkpoint_step_*.pt")) if ".rank" not in f and ".tmp" not in f]
    for f in sorted(files, key=lambda f: int(f.rsplit("_", 1)[1].split(".")[0]), reverse=True):
        if is_complete(f):
            return f
    return None
