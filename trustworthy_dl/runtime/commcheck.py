"""RCCL-semantics replay of a run's communication: does the issue order deadlock under RCCL?

The multi-rank tests run on gloo (CPU).  gloo is more permissive than RCCL: a gloo ``isend`` to one
peer proceeds independently of a receive from another, while RCCL runs every operation of a
communicator in issue order on that communicator's stream, starts the operations of one
``batch_isend_irecv`` group together, and orders operations across communicators only through the
compute stream (an operation waits for the compute work enqueued before it; compute enqueued after
``work.wait()`` waits for that operation).  A schedule that passes on gloo can therefore hang on
RCCL — the classic case is a send to one neighbour queued on a communicator ahead of a receive from
the other.  Nothing in the reference addresses this (its "distributed" trainer never communicates
between stages: /root/reference/distributed_trainer.py:161, 182).

``CommRecorder`` (enabled with ``TDL_COMMCHECK=<dir>``) records, per rank and in issue order, every
P2P group (peer, direction, bytes), every collective (name, bytes, members), every ``wait()`` on
their works and the c10d-store reveals (``set`` / ``get`` keys: a ``get`` blocks the host until the
key's ``set``).  ``replay`` simulates the recorded ranks under the RCCL model:

* communicators: a collective or a ``batch_isend_irecv`` group runs on its process group's
  communicator, an unbatched ``isend`` / ``irecv`` on the 2-rank communicator of (group, pair);
* a rank's HOST moves through its events in order and is blocked only by a store ``get`` (until
  some host passed the key's ``set``) and by a host sync (``note_host_sync``: a device->host read,
  until every operation the rank waited on before it completed) — ``wait()`` itself is stream
  ordered and does not block the host;
* an operation can START once its rank's host issued it, the previous operation on the same
  communicator completed, and every operation the rank waited on before issuing it completed;
* a P2P group COMPLETES when, for each of its sends / receives, the matching receive / send (the
  k-th one between the two ranks on that communicator) belongs to a STARTED group, with equal bytes;
* a collective completes when the matching collective (k-th on the communicator) of every member
  started, with equal names and bytes.

Anything left incomplete is a deadlock (or a mismatch), reported with the blocked heads."""
from __future__ import annotations

import atexit
import json
import os
import threading
from collections import defaultdict
from typing import Dict, List, Optional

import torch.distributed as dist


def _pg_name(group) -> str:
    if group is None or group is dist.GroupMember.WORLD:
        return "world"
    name = getattr(group, "group_name", None)
    if name:
        return str(name)
    return "pg:" + ",".join(str(r) for r in dist.get_process_group_ranks(group))


def _members(group) -> List[int]:
    if group is None or group is dist.GroupMember.WORLD:
        return list(range(dist.get_world_size()))
    return list(dist.get_process_group_ranks(group))


def _nbytes(t) -> int:
    return int(t.numel() * t.element_size())


class _Work:
    """Proxy of a c10d work that records its ``wait``."""

    def __init__(self, work, rec: "CommRecorder", op_id: int):
        self._w, self._rec, self._id = work, rec, op_id

    def wait(self, *a, **k):
        self._rec.events.append({"wait": self._id})
        return self._w.wait(*a, **k)

    def __getattr__(self, name):
        return getattr(self._w, name)


class _Store:
    """Proxy of the c10d store that records ``set`` / ``get``."""

    def __init__(self, store, rec: "CommRecorder"):
        self._s, self._rec = store, rec

    def set(self, key, value):
        if threading.current_thread() is threading.main_thread():   # not the watchdog / heartbeat threads
            self._rec.events.append({"store_set": str(key)})
        return self._s.set(key, value)

    def get(self, key):
        v = self._s.get(key)
        if threading.current_thread() is threading.main_thread():
            self._rec.events.append({"store_get": str(key)})
        return v

    def __getattr__(self, name):
        return getattr(self._s, name)


class CommRecorder:
    def __init__(self, out_dir: str):
        self.out_dir = out_dir
        self.events: List[Dict] = []
        self._n = 0
        self._orig: Dict[str, object] = {}

    # ---------------------------------------------------------------- recording
    def _issue(self, ev: Dict) -> int:
        ev["id"] = self._n
        self._n += 1
        self.events.append(ev)
        return ev["id"]

    def install(self):
        c10d = dist.distributed_c10d
        rec = self
        orig_batch = dist.batch_isend_irecv

        def batch_isend_irecv(ops):
            me = dist.get_rank()
            groups = {_pg_name(p.group) for p in ops}
            assert len(groups) == 1, "one communicator per batch"
            items = [("send" if p.op.__name__ == "isend" else "recv", int(p.peer), _nbytes(p.tensor)) for p in ops]
            oid = rec._issue({"kind": "p2p", "pg": groups.pop(), "rank": me, "ops": items})
            return [_Work(w, rec, oid) for w in orig_batch(ops)]

        def wrap_coll(name, fn, tensor_arg=0):
            def inner(*args, **kw):
                group = kw.get("group")
                if group is None:
                    # positional group argument of the wrapped collectives
                    pos = {"all_gather_into_tensor": 2, "broadcast": 2, "all_reduce": 2, "barrier": 0,
                           "reduce_scatter_tensor": 3, "all_gather": 2}.get(name)
                    if pos is not None and len(args) > pos and not isinstance(args[pos], (int, float)):
                        group = args[pos]
                t = args[tensor_arg] if name != "barrier" and args else None
                nb = _nbytes(t) if hasattr(t, "numel") else 0
                oid = rec._issue({"kind": "coll", "name": name, "pg": _pg_name(group), "bytes": nb,
                                  "members": _members(group)})
                w = fn(*args, **kw)
                if kw.get("async_op"):
                    return _Work(w, rec, oid)
                rec.events.append({"wait": oid})
                if name in ("all_gather_object", "barrier"):
                    rec.events.append({"host_sync": True})   # objects are read on the host
                return w
            return inner

        for name in ("all_gather_into_tensor", "broadcast", "all_reduce", "barrier", "reduce_scatter_tensor",
                     "all_gather", "all_gather_object"):
            fn = getattr(dist, name)
            self._orig[name] = fn
            setattr(dist, name, wrap_coll(name, fn))
        self._orig["batch_isend_irecv"] = orig_batch
        dist.batch_isend_irecv = batch_isend_irecv
        # the async 1F1B schedule's unbatched sends / receives (parallel/comm.py isend / irecv)
        from ..parallel import comm as p2p

        def single(kind, fn):
            def inner(t, peer, group=None):
                me = dist.get_rank()
                lo, hi = min(me, int(peer)), max(me, int(peer))
                # an unbatched P2P op runs on the 2-rank communicator of (group, pair)
                oid = rec._issue({"kind": "p2p", "pg": f"{_pg_name(group)}|{lo}-{hi}", "rank": me,
                                  "ops": [(kind, int(peer), _nbytes(t))]})
                return _Work(fn(t, peer, group=group), rec, oid)
            return inner
        self._orig["comm.isend"], self._orig["comm.irecv"] = p2p.isend, p2p.irecv
        p2p.isend, p2p.irecv = single("send", p2p.isend), single("recv", p2p.irecv)
        orig_store = c10d._get_default_store
        self._orig["_get_default_store"] = orig_store
        c10d._get_default_store = lambda: _Store(orig_store(), rec)
        atexit.register(self.dump)
        return self

    def uninstall(self):
        c10d = dist.distributed_c10d
        from ..parallel import comm as p2p
        for name, fn in self._orig.items():
            if name == "_get_default_store":
                c10d._get_default_store = fn
            elif name.startswith("comm."):
                setattr(p2p, name[5:], fn)
            else:
                setattr(dist, name, fn)
        self._orig = {}

    def dump(self, path: Optional[str] = None):
        if not self.events:
            return
        try:
            rank = dist.get_rank() if dist.is_initialized() else int(os.environ.get("RANK", "0"))
        except Exception:
            rank = int(os.environ.get("RANK", "0"))
        os.makedirs(self.out_dir, exist_ok=True)
        with open(path or os.path.join(self.out_dir, f"rank{rank}.json"), "w") as f:
            json.dump(self.events, f)


_REC: Optional[CommRecorder] = None


def note_host_sync(device: bool = False):
    """Mark a device->host synchronisation of this rank: the host blocks until every operation it
    waited on so far has completed (``device``: a whole-device synchronize, until every operation it
    issued so far has).  No-op unless the recorder is installed."""
    if _REC is not None and threading.current_thread() is threading.main_thread():
        _REC.events.append({"host_sync": True, "device": bool(device)})


def maybe_install() -> Optional[CommRecorder]:
    """Install the recorder once per process when ``TDL_COMMCHECK`` names an output directory."""
    global _REC
    d = os.environ.get("TDL_COMMCHECK")
    if d and _REC is None:
        _REC = CommRecorder(d).install()
    return _REC


# -------------------------------------------------------------------- replay under the RCCL model
def replay(events_by_rank: Dict[int, List[Dict]]) -> Dict:
    """Simulate the recorded ranks under the RCCL model (module docstring).  Returns
    {"ok": bool, "ops": total, "completed": n, "blocked": [...], "mismatches": [...]}."""
    ops: Dict[tuple, Dict] = {}                 # (rank, id) -> op
    order: Dict[int, List[int]] = {}
    waits: Dict[int, List[tuple]] = {}          # per rank: waited ops in wait order
    seq: Dict[int, List[Dict]] = {}             # per rank: host-side events in order
    for r, evs in events_by_rank.items():
        last_on_pg: Dict[str, int] = {}
        w: List[tuple] = []
        ids: List[int] = []
        sq: List[Dict] = []
        for ev in evs:
            if "wait" in ev:
                w.append((r, ev["wait"]))
            elif "store_set" in ev or "store_get" in ev:
                sq.append(dict(ev))
            elif "host_sync" in ev:
                sq.append({"host_sync": True, "nw": len(w), "upto": [(r, j) for j in ids] if ev.get("device") else []})
            else:
                i = ev["id"]
                fifo = (r, last_on_pg[ev["pg"]]) if ev["pg"] in last_on_pg else None
                last_on_pg[ev["pg"]] = i
                ops[(r, i)] = dict(ev, rank=r, fifo=fifo, nw=len(w))
                sq.append({"issue": (r, i)})
                ids.append(i)
        order[r], waits[r], seq[r] = ids, w, sq
    # matching: the k-th send r->p on a communicator pairs with the k-th recv at p from r on it;
    # the k-th collective on a communicator pairs across its members
    pairs: Dict[tuple, List[tuple]] = defaultdict(list)
    colls: Dict[tuple, List[tuple]] = defaultdict(list)
    for r in sorted(order):
        for i in order[r]:
            op = ops[(r, i)]
            if op["kind"] == "p2p":
                for d, peer, nb in op["ops"]:
                    src, dst = (r, peer) if d == "send" else (peer, r)
                    pairs[(op["pg"], src, dst, d)].append(((r, i), nb))
            else:
                colls[(op["pg"], r)].append((r, i))
    mismatches = []
    partner: Dict[tuple, List] = defaultdict(list)
    for (pg, src, dst, d), lst in pairs.items():
        other = pairs.get((pg, src, dst, "recv" if d == "send" else "send"), [])
        if d == "send" and len(other) != len(lst):
            mismatches.append({"pg": pg, "src": src, "dst": dst, "sends": len(lst), "recvs": len(other)})
        for k, (key, nb) in enumerate(lst):
            if k < len(other):
                okey, onb = other[k]
                if d == "send" and onb != nb:
                    mismatches.append({"pg": pg, "src": src, "dst": dst, "k": k, "send_bytes": nb, "recv_bytes": onb})
                partner[key].append(okey)
            else:
                partner[key].append(None)
    for (pg, r), lst in colls.items():
        for k, key in enumerate(lst):
            op = ops[key]
            for m in op["members"]:
                if m == r:
                    continue
                other = colls.get((pg, m), [])
                if k >= len(other):
                    partner[key].append(None)
                    continue
                o = ops[other[k]]
                if o["name"] != op["name"] or o["bytes"] != op["bytes"]:
                    mismatches.append({"pg": pg, "k": k, "rank": r, "peer": m, "op": op["name"], "peer_op": o["name"],
                                       "bytes": op["bytes"], "peer_bytes": o["bytes"]})
                partner[key].append(other[k])
    host = {r: 0 for r in seq}                  # next host event of each rank
    issued, started, done = set(), set(), set()
    keys_set: set = set()
    wdone = {r: 0 for r in seq}                 # longest prefix of the rank's waits that completed
    progress = True
    while progress:
        progress = False
        for r, sq in seq.items():               # hosts advance until a blocking event
            while host[r] < len(sq):
                e = sq[host[r]]
                if "store_get" in e and e["store_get"] not in keys_set:
                    break
                if "host_sync" in e and (wdone[r] < e["nw"] or not all(k in done for k in e["upto"])):
                    break
                if "store_set" in e:
                    keys_set.add(e["store_set"])
                if "issue" in e:
                    issued.add(e["issue"])
                host[r] += 1
                progress = True
        for key in issued - started:            # stream / communicator order
            op = ops[key]
            if (op["fifo"] is None or op["fifo"] in done) and wdone[key[0]] >= op["nw"]:
                started.add(key)
                progress = True
        for key in started - done:
            if all(p is not None and p in started for p in partner[key]):
                done.add(key)
                progress = True
        for r, w in waits.items():
            while wdone[r] < len(w) and w[wdone[r]] in done:
                wdone[r] += 1
                progress = True
    blocked = []
    for r in sorted(seq):
        pending = [i for i in order[r] if (r, i) not in done]
        if pending or host[r] < len(seq[r]):
            item = {"rank": r, "host_blocked_on": seq[r][host[r]] if host[r] < len(seq[r]) else None}
            if pending:
                op = ops[(r, pending[0])]
                item.update(id=pending[0], kind=op["kind"], pg=op["pg"], ops=op.get("ops") or op.get("name"),
                            issued=(r, pending[0]) in issued, started=(r, pending[0]) in started)
            blocked.append(item)
    return {"ok": not blocked and not mismatches, "ops": len(ops), "completed": len(done),
            "blocked": blocked, "mismatches": mismatches[:20]}


def replay_dir(d: str) -> Dict:
    evs = {}
    for fn in sorted(os.listdir(d)):
        if fn.startswith("rank") and fn.endswith(".json"):
            with open(os.path.join(d, fn)) as f:
                evs[int(fn[4:-5])] = json.load(f)
    return replay(evs)


if __name__ == "__main__":
    import sys
    res = replay_dir(sys.argv[1])
    print(json.dumps(res, indent=1))
    sys.exit(0 if res["ok"] else 1)
