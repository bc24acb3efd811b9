"""Distributed audit protocol of ``PipelineEngine`` (one process per stage): commit, private key,
sketches, private opening through the c10d store; applied gradient, opened contributions, inputs
and input gradients over P2P; verification on the auditor's live optimizer mirror.

Ordering is what makes it binding, so the small messages go host to host through the store: an
auditor reveals its key only after ``store.get`` returned the commitments, and its opened set only
after it returned the sketches — nothing the auditee sends after a reveal can change what it had
committed before it (a P2P send is only enqueued when the host posts it; the auditor could not tell
when it landed without a device sync).  Store payloads are JSON (an auditee's bytes are never
unpickled).  Every rank runs the phases in the same order — all auditee "commit" posts, then all
auditor "key" posts, ... — so no store read waits on a phase that waits on it.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..runtime.commcheck import note_host_sync
from ..security import stage_verifier as SV


def _enc_json(obj) -> str:
    return json.dumps(obj, separators=(",", ":"))


class DistAuditMixin:
    """Distributed audit protocol (mixed into ``PipelineEngine``)."""

    def _tensor_root(self, t: torch.Tensor) -> torch.Tensor:
        """Merkle root of a tensor's bytes (16-bit tensors hashed as pairs of elements)."""
        from ..security.grad_audit import merkle_root
        t = t.detach().contiguous().reshape(-1)
        if t.element_size() == 4:
            return merkle_root(t)
        if t.element_size() == 2 and t.numel() % 2 == 0:
            return merkle_root(t.view(torch.int32))
        return merkle_root(t.float())

    def _list_row(self, ts: List[torch.Tensor]) -> torch.Tensor:
        """hash_row of the root over the roots of a list of tensors (digest cross-checks)."""
        from ..security.grad_audit import hash_row, merkle_root
        roots = torch.stack([self._tensor_root(t) for t in ts])
        return hash_row(merkle_root(roots.reshape(-1)))

    def _audit_dist(self, rows: Dict[int, torch.Tensor]):
        """One rank's part of the step's audit (stage s of S; auditee of its auditor, auditor of its
        previous stage and — as the stage before the loss stage — of the loss stage).

        Mirror mode (backward audit, commitments on):
          1. commit   (auditee) store: Merkle roots of the M contributions, the applied gradient and
                      the master weights (+ public running sketches for the targeted audit); P2P on
                      the audit communicator: the applied gradient (and, when its auditor's mirror
                      is not seeded for this plan, the optimizer state);
          2. key      (auditor) after reading the commitments: a private 63-bit sketch key;
          3. sketches (auditee) the M keyed contribution sketches;
          4. open     (auditor) after reading the sketches: whether to audit (``audit_prob``) and
                      which ``audit_micro_k`` micro-batches (+ the targeted one, opt-in);
          5. ship     (auditee, P2P) the opened contributions; for non-first, non-loss stages also
                      the inputs and the input gradients it sent upstream for them;
          6. verify   (auditor, on its mirror) ``_verify_applied`` every step, ``_audit_one`` per
                      opened micro-batch; its upstream neighbour and it put the roots of the
                      inputs / input gradients sent, received and shipped into the digest, compared
                      on every rank (``_audit_vectors``).
        Weight-shipping mode (data-parallel replicas, forward-only audit): 4-6 with the stage's
        bf16 weights shipped (``_audit_early_ship``) instead of a mirror."""
        st = self.my_stage()
        if st is None:
            return
        me = self.rank
        s, S = st.stage_id, self.plan.num_stages
        prev, nxt = self.comm.prev, self.comm.next
        bwd = self.cfg.audit_backward
        act_g, grad_g = (self._dir_groups if self.p2p_mode == "async" else (None, None))
        M = len(self._audit_batch)
        d = rows[me]
        mirror = bool(self._gsk_on)
        if self._audit_rng is None:
            seed = self.cfg.monitor_seed
            self._audit_rng = __import__("random").Random(
                int.from_bytes(os.urandom(8), "little") if seed is None else seed * 7919 + me)
        store = dist.distributed_c10d._get_default_store()
        tag = f"tdl_audit/{self.plan.version}/{self.global_step}"
        # my auditees: prev (I am its next stage), and nxt when it is the loss stage
        peers = []
        if prev is not None:
            peers.append((prev, s - 1, False))
        if bwd and nxt is not None and s + 1 == S - 1:
            peers.append((nxt, s + 1, True))
        # my auditor: nxt, or prev when I am the loss stage
        my_auditor = nxt if nxt is not None else (prev if bwd and s == S - 1 and prev is not None else None)
        mirs = {p: self._audit_mirror(tuple(self.plan.ranges[sid]), sid) for p, sid, _ in peers}
        a_cost = self._audit_cost

        # ---- 1. commit (auditee): roots through the store, the applied gradient over P2P
        p2p_ops, seed_ops = [], []
        if mirror and my_auditor is not None:
            C = self._contrib_commitments(me, st)
            G = self._applied_gradient(me, st)
            run = self._gsk_run.get(me) if self._targeted else None
            mark = (self.plan.version, tuple(st.layer_range), self._mirror_epoch)
            note_host_sync()
            payload = {"C": C.cpu().tolist(), "step_count": st.flat.step_count,
                       "run": run.cpu().tolist() if run is not None else None}
            store.set(f"{tag}/com/{me}", _enc_json(payload))
            p2p_ops.append(("send", G.contiguous(), my_auditor))
            if self._seed_mark != mark:
                master, m1, m2, _ = self._optimizer_state(me, st)
                seed_ops += [("send", t.contiguous(), my_auditor) for t in (master, m1, m2)]
                self._seed_mark = mark
        seeding: Dict[int, bool] = {}
        if mirror:
            for p, _, _ in peers:
                mir = mirs[p]
                g_in = getattr(mir, "_g_in", None)
                if g_in is None or g_in.numel() != mir.flat.numel:
                    g_in = mir._g_in = torch.empty(mir.flat.numel, dtype=torch.float32, device=self.device)
                p2p_ops.append(("recv", g_in, p))
                seeding[p] = not self._mirror_seeded(mir)
                if seeding[p]:
                    seed_ops += [("recv", t, p) for t in (mir.flat.master, mir.flat.exp_avg, mir.flat.exp_avg_sq)]
        work = None
        if p2p_ops or seed_ops:
            g = self._audit_pg
            allops = p2p_ops + seed_ops
            ops = [dist.P2POp(dist.isend if k == "send" else dist.irecv, t, r, g) for k, t, r in allops]
            nbytes = lambda lst, kind=None: sum(t.numel() * t.element_size() for k, t, _ in lst  # noqa: E731
                                                if kind is None or k == kind)
            a_cost["bytes"] += nbytes(p2p_ops)
            a_cost["sent"] += nbytes(p2p_ops, "send")
            a_cost["seed_bytes"] += nbytes(seed_ops, "recv")
            self._note_peers([(t, r) for k, t, r in allops if k == "send"],
                             [(t, r) for k, t, r in allops if k == "recv"], "audit")
            work = dist.batch_isend_irecv(ops)

        # ---- 2. key (auditor): only after the commitments were read; for a tie-group member also
        # this auditor's part of the step's shared tie key
        got: Dict[int, dict] = {}
        keys: Dict[int, int] = {}
        tie_pos = self._tie_members() if mirror else []
        for k in self._tkey_trash:      # last step's tie-key parts: every rank read them before it
            store.delete_key(k)         # joined that step's digest all-gather
        self._tkey_trash = []
        if mirror:
            for p, sid, _ in peers:
                k = f"{tag}/com/{p}"
                got[p] = json.loads(store.get(k).decode())
                store.delete_key(k)
                keys[p] = self._audit_rng.getrandbits(63)
                store.set(f"{tag}/key/{p}", str(keys[p]))
                if sid in tie_pos:
                    k = f"{tag}/tkey/{p}"
                    store.set(k, str(self._audit_rng.getrandbits(63)))
                    self._tkey_trash.append(k)

        def tie_key():
            parts = [int(store.get(f"{tag}/tkey/{self.plan.ranks[j]}").decode()) for j in tie_pos]
            return self._tie_key_of(parts)

        # ---- 3. sketches (auditee)
        if mirror and my_auditor is not None:
            k = f"{tag}/key/{me}"
            key_req = int(store.get(k).decode())
            store.delete_key(k)
            sT = self._tie_sketches(me, st, tie_key()) if s in tie_pos else None
            note_host_sync()
            sk = self._contrib_sketches(me, st, key_req).cpu().tolist()
            store.set(f"{tag}/sk/{me}", _enc_json({"s": sk, "t": sT.cpu().tolist() if sT is not None else None}))

        # ---- 4. open (auditor): only after the sketches were read
        sketches: Dict[int, Optional[torch.Tensor]] = {}
        tsk: Dict[int, Optional[torch.Tensor]] = {}
        tkey = tie_key() if any(sid in tie_pos for _, sid, _ in peers) else None
        if mirror:
            for p, _, _ in peers:
                k = f"{tag}/sk/{p}"
                pl = json.loads(store.get(k).decode())
                store.delete_key(k)
                pl = pl if isinstance(pl, dict) else {}
                sketches[p] = self._as_tensor(pl.get("s"), torch.float32)
                t = self._as_tensor(pl.get("t"), torch.float32) if pl.get("t") is not None else None
                from ..security.grad_audit import K_KEYED
                tsk[p] = t if t is not None and t.dim() == 2 and tuple(t.shape) == (M, K_KEYED) else None
        tgt: Dict[int, int] = {}
        if self._targeted and peers:
            zs = []
            for p, sid, nxt_peer in peers:
                ys = [self._output_stat(self._audit_inputs[m]) for m in range(M)] if (not nxt_peer and sid >= 0) else None
                run = got.get(p, {}).get("run") if mirror else None
                run = self._as_tensor(run, torch.float32) if run is not None else None
                zs.append(self._target_scores(ys, run))
            vals = [torch.stack([z.max(), z.argmax().float()]) if z is not None else
                    torch.tensor([-1.0, -1.0], device=self.device) for z in zs]
            note_host_sync()
            vals = torch.stack(vals).tolist()
            for (p, _, _), (zm, i) in zip(peers, vals):
                tgt[p] = int(i) if zm > self.cfg.audit_target_z else -1
            self._target_log.extend((self.global_step, p, m) for p, m in tgt.items() if m >= 0)

        def choose(extra):
            if self.cfg.audit_prob < 1.0 and self._audit_rng.random() >= self.cfg.audit_prob:
                return [extra] if extra >= 0 else []
            kk = max(1, min(int(self.cfg.audit_micro_k), M))
            return list(dict.fromkeys(self._audit_rng.sample(range(M), kk) + ([extra] if extra >= 0 else [])))

        def enc(ms):
            return ",".join(str(m) for m in ms) if ms else "-1"

        def dec(v):
            return [int(t) for t in v.decode().split(",") if int(t) >= 0]
        opened: Dict[int, List[int]] = {}
        for p, sid, nxt_peer in peers:
            opened[p] = choose(tgt.get(p, -1)) if self._audit_now else []
            store.set(f"{tag}/req/{p}", enc(opened[p]))
            if not nxt_peer and sid > 0 and bwd:
                store.set(f"{tag}/reqh/{p}", enc(opened[p]))   # for p's upstream stage: x / dx roots
        ms_req: List[int] = []
        if my_auditor is not None:
            k = f"{tag}/req/{me}"
            ms_req = dec(store.get(k))
            store.delete_key(k)
        # as the upstream neighbour of nxt (when nxt is not the loss stage): roots of the outputs I
        # sent it and of the input gradients I received from it, for the micro-batches its auditor opened
        for slot in (SV.D_DXHASH_RECV, SV.D_XHASH_SENT):
            d[slot:slot + 8].fill_(-1.0)
        if bwd and nxt is not None and s + 1 < S - 1:
            k = f"{tag}/reqh/{nxt}"
            mh = dec(store.get(k))
            store.delete_key(k)
            if mh and all(m in self._audit_recv_dy for m in mh):
                d[SV.D_DXHASH_RECV:SV.D_DXHASH_RECV + 8].copy_(self._list_row([self._audit_recv_dy[m] for m in mh]))
            if mh and all(m in self._audit_outputs for m in mh):
                d[SV.D_XHASH_SENT:SV.D_XHASH_SENT + 8].copy_(self._list_row([self._audit_outputs[m] for m in mh]))

        # ---- 5. ship (auditee) / receive (auditor)
        x_send, dx_send = [], []
        if ms_req and 0 < s < S - 1:
            x_send = [self._audit_inputs[m].contiguous() for m in ms_req]
            if bwd and all(m in self._audit_sent_dx for m in ms_req):
                dx_send = [self._audit_sent_dx[m].contiguous() for m in ms_req]
            store.set(f"{tag}/shape/{me}", ",".join(str(v) for v in x_send[0].shape))
        early = self._early_ship
        self._early_ship = None
        sends, recvs = [], []
        if ms_req:
            if not mirror and early is None:
                sends.append((st.flat.data, my_auditor))
            sends += [(t, my_auditor) for t in x_send]
            sends += [(t, my_auditor) for t in dx_send]
            if mirror:
                sends += [(t.contiguous(), my_auditor) for t in self._open_contributions(me, st, ms_req)]
        inbound: Dict[int, dict] = {}
        for p, sid, nxt_peer in peers:
            ms = opened[p]
            ib = inbound[p] = {"x": [], "dx": [], "c": []}
            if not ms:
                continue
            mir = mirs[p]
            if not mirror and early is None:
                recvs.append((mir.flat.data, p))
            if not nxt_peer and sid > 0:
                k = f"{tag}/shape/{p}"
                shape = torch.Size([int(v) for v in store.get(k).decode().split(",")])
                store.delete_key(k)
                ib["x"] = [torch.empty(shape, dtype=self.dtype, device=self.device) for _ in ms]
                recvs += [(t, p) for t in ib["x"]]
                if bwd:
                    ib["dx"] = [torch.empty(shape, dtype=self.dtype, device=self.device) for _ in ms]
                    recvs += [(t, p) for t in ib["dx"]]
            if mirror:
                ib["c"] = [torch.empty(mir.flat.numel, dtype=torch.float32, device=self.device) for _ in ms]
                recvs += [(t, p) for t in ib["c"]]
        self._audit_transfer(sends, recvs, prev, nxt, act_g, grad_g)
        if work is not None:
            for w in work:
                w.wait()
        if early is not None:
            for w in early[0]:
                w.wait()

        # ---- 6. verify (auditor)
        d[SV.D_WHASH_PREV:SV.D_WHASH_PREV + 8].fill_(-1.0)
        d[SV.D_WHASH_NEXT:SV.D_WHASH_NEXT + 8].fill_(-1.0)
        d[SV.D_DXHASH_SHIP:SV.D_DXHASH_SHIP + 8].fill_(-1.0)
        d[SV.D_XHASH_SHIP:SV.D_XHASH_SHIP + 8].fill_(-1.0)
        from ..security.grad_audit import hash_row, merkle_root
        for p, sid, nxt_peer in peers:
            mir = mirs[p]
            ms, ib = opened[p], inbound[p]
            res = None
            C = s_p = key = None
            if mirror:
                if seeding[p]:
                    self._seed_mirror(mir, None, None, None, int(got[p].get("step_count", 0)))
                C = self._as_tensor(got[p]["C"], torch.int32)
                s_p, key = sketches[p], keys[p]
                if C is None or s_p is None or s_p.dim() != 2 or s_p.shape[0] != M:
                    one = torch.ones(1, device=self.device)
                    res = (one, one * (SV.AK_GAPP + SV.AK_WHASH), one * 1e30)
                    C = s_p = None
                else:
                    kd, e = self._verify_applied(mir, C, mir._g_in, s_p, key)
                    res = ((kd > 0).float(), kd, e)
                if sid in tie_pos:
                    self._write_tie(d, mir, mir._g_in, tsk.get(p), tkey, next_slot=nxt_peer)
                self._mirror_pending.append((mir, mir._g_in, p))
                d[SV.D_MIRROR:SV.D_MIRROR + 1].fill_(1.0)
                slot = SV.D_SUMSQ_NEXT if nxt_peer else SV.D_SUMSQ_PREV
                d[slot:slot + 1].copy_(mir.clip_sumsq(mir._g_in).reshape(1))
            for j, m in enumerate(ms):
                if nxt_peer:
                    labels = self._audit_targets[m].to(self.device, non_blocking=True)
                    r1 = self._audit_one(mir, self._audit_outputs.get(m), m, M, labels=labels,
                                         dx_seen=self._audit_recv_dy.get(m), c_m=ib["c"][j] if ib["c"] else None,
                                         C=C, s=s_p, key=key, sT=tsk.get(p), tkey=tkey)
                else:
                    xp = ib["x"][j] if ib["x"] else self._stage_input(self._audit_batch[m], mir)
                    dy = self._audit_sent_dx.get(m) if bwd else None
                    r1 = self._audit_one(mir, xp, m, M, y_seen=self._audit_inputs[m], dy=dy,
                                         dx_seen=ib["dx"][j] if ib["dx"] else None,
                                         c_m=ib["c"][j] if ib["c"] else None, C=C, s=s_p, key=key,
                                         sT=tsk.get(p), tkey=tkey)
                res = self._combine(res, r1)
            if res is not None:
                self._write_verdict(d, res, next_slot=nxt_peer)
            if not mirror and ms:
                slot = SV.D_WHASH_NEXT if nxt_peer else SV.D_WHASH_PREV
                d[slot:slot + 8].copy_(hash_row(merkle_root(mir.flat.data.view(torch.int32)
                                                            if mir.flat.data.element_size() == 2 and mir.flat.numel % 2 == 0
                                                            else mir.flat.data.float())))
            if not nxt_peer and ib["x"]:
                d[SV.D_XHASH_SHIP:SV.D_XHASH_SHIP + 8].copy_(self._list_row(ib["x"]))
            if not nxt_peer and ib["dx"]:
                d[SV.D_DXHASH_SHIP:SV.D_DXHASH_SHIP + 8].copy_(self._list_row(ib["dx"]))
        self._audit_inputs = {}
        self._audit_sent_dx = {}
        self._audit_recv_dy = {}
        self._audit_outputs = {}

    @torch.no_grad()
    def _heal_dist(self, nodes: List[int]):
        """Distributed counterpart of ``_heal_from_mirror``, run by every rank from the same lagged
        host report (so the same steps and list on every rank): for each node whose committed master
        weights failed its auditor's mirror check, the auditor ships its mirror's verified optimizer
        state (master, AdamW moments) and the stage adopts it (compute weights rebuilt, integrity
        checksum re-baselined).  Both sides are post-update at the same step, so the next commitment
        matches.  A rank that refuses keeps failing the check (and is compromised)."""
        S = self.plan.num_stages
        me = self.rank
        sends, recvs, adopt = [], [], None
        for x in nodes:
            sid = self.plan.stage_of_rank(x)
            if sid is None or S < 2:
                continue
            aud = self.plan.ranks[sid + 1] if sid + 1 < S else self.plan.ranks[sid - 1]
            if me == aud:
                mir = self._audit_mirror(tuple(self.plan.ranges[sid]), sid)
                if self._mirror_seeded(mir):
                    sends += [(t, x) for t in (mir.flat.master, mir.flat.exp_avg, mir.flat.exp_avg_sq)]
            elif me == x:
                st = self.my_stage()
                # the auditor ships only from a mirror seeded in the current epoch, which is when this
                # stage shipped it a seed in this epoch: both sides decide alike
                if st is not None and self._seed_mark == (self.plan.version, tuple(st.layer_range), self._mirror_epoch):
                    recvs += [(t, aud) for t in (st.flat.master, st.flat.exp_avg, st.flat.exp_avg_sq)]
                    adopt = st
        if not sends and not recvs:
            return
        g = self._audit_pg
        self._note_peers(sends, recvs, "audit")
        ops = [dist.P2POp(dist.isend, t.contiguous(), r, g) for t, r in sends] + \
              [dist.P2POp(dist.irecv, t, r, g) for t, r in recvs]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        self._audit_cost["seed_bytes"] += sum(t.numel() * t.element_size() for t, _ in recvs)
        self._audit_cost["heals"] = self._audit_cost.get("heals", 0) + (1 if adopt is not None else 0)
        if adopt is not None:
            f = adopt.flat
            if f.data is not f.master:
                f.data.copy_(f.master)
            from ..ops.layers import bump_weight_generation
            bump_weight_generation()
            adopt.param_checksum = None      # re-baselined at the next step's integrity check

    def _as_tensor(self, v, dtype) -> Optional[torch.Tensor]:
        """A JSON payload from a peer as a device tensor (None if it is not a rectangular number list)."""
        try:
            t = torch.tensor(v, dtype=torch.int64 if dtype == torch.int32 else dtype)
        except (TypeError, ValueError, RuntimeError):
            return None
        if dtype == torch.int32:
            t = ((t & 0xFFFFFFFF) - ((t & 0x80000000) << 1)).to(torch.int32)
        return t.to(self.device)
