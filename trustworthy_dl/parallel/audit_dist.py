"""Distributed recompute-audit protocol of ``PipelineEngine`` (one process per stage): commit,
private reveal through the c10d store, ship, verify on a mirror of the audited stage.
"""
from __future__ import annotations

import os
from typing import Dict, List

import torch
import torch.distributed as dist

from ..runtime.commcheck import note_host_sync
from ..security import stage_verifier as SV


class DistAuditMixin:
    """Distributed audit protocol (mixed into ``PipelineEngine``)."""

    def _audit_dist(self, rows: Dict[int, torch.Tensor]):
        """Distributed audit protocol of one rank (stage s of S):

        1. commit: every audited stage sends the exact hashes of its running gradient after every
           micro-batch (one [M+1] int64 tensor; CommitmentMixin) to its auditor BEFORE any choice is
           revealed;
        2. reveal: each auditor draws privately whether to audit, which ``audit_micro_k``
           micro-batches and a 63-bit sketch key, and posts them in the c10d store (host to host, no
           device sync); the auditee reads them only now, after every output and gradient of the
           step reached its peers and its commitments went out;
        3. ship: the auditee sends its bf16 weights, (non-first, non-loss stages) its input and the
           input gradient it sent upstream for those micro-batches, and its answers: the keyed
           sketch of each audited micro-batch's committed contribution plus the re-computed hashes of
           the snapshots it came from (``_answer_challenge``); the loss stage ships only its weights
           and answers (its auditor holds its input, the labels and the gradient it sent);
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
        if self._audit_rng is None:
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
        # ---- 1. commitments: exact running-gradient hashes (and, for targeting, the public running
        # sketches) to my auditor before any reveal
        runs_in: Dict[int, torch.Tensor] = {}
        coms_in: Dict[int, torch.Tensor] = {}
        keyed = bool(bwd and self._gsk_on)
        if keyed:
            c_send, c_recv = [], []
            if my_auditor is not None:
                c_send.append((self._gcom[self.rank], my_auditor))
                if self._targeted:
                    c_send.append((self._gsk_run[self.rank], my_auditor))
            for peer, on in ((prev, audit_prev), (nxt, audit_next)):
                if on:
                    coms_in[peer] = torch.empty(M + 1, dtype=torch.int64, device=self.device)
                    c_recv.append((coms_in[peer], peer))
                    if self._targeted:
                        runs_in[peer] = torch.empty(M + 1, 2, dtype=torch.float32, device=self.device)
                        c_recv.append((runs_in[peer], peer))
            self._audit_transfer(c_send, c_recv, prev, nxt, act_g, grad_g)
        # the auditees' last commitments as received here: compared on every rank with what each
        # auditee reports for itself (``_gsk_mismatch``)
        from ..security.grad_audit import fold_hash64
        for peer, slot in ((prev, SV.D_GCOM_RECV_PREV), (nxt, SV.D_GCOM_RECV_NEXT)):
            com = coms_in.get(peer) if peer is not None else None
            if com is not None:   # + 1: a zeroed slot (no audit this step) reads as "none"
                d[slot:slot + 2].copy_(fold_hash64(com[-1]) + 1.0)
            else:
                d[slot:slot + 2].fill_(0.0)

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
            self._target_log.extend((self.global_step, n, m) for n, m in ((prev, tgt_prev), (nxt, tgt_next)) if m >= 0)

        def choose(extra):
            if self.cfg.audit_prob < 1.0 and self._audit_rng.random() >= self.cfg.audit_prob:
                return [extra] if extra >= 0 else []
            k = max(1, min(int(self.cfg.audit_micro_k), M))
            return list(dict.fromkeys(self._audit_rng.sample(range(M), k) + ([extra] if extra >= 0 else [])))
        ms_prev = choose(tgt_prev) if audit_prev else []
        ms_next = choose(tgt_next) if audit_next else []
        key_prev, key_next = self._audit_rng.getrandbits(63), self._audit_rng.getrandbits(63)

        def enc(ms, key=None):
            v = ",".join(str(m) for m in ms) if ms else "-1"
            return v if key is None else f"{v};{key}"

        def dec(v):
            return [int(t) for t in v.decode().split(";")[0].split(",") if int(t) >= 0]
        if audit_prev:
            store.set(f"{tag}/req/{prev}", enc(ms_prev, key_prev))
            if s - 1 > 0 and bwd:
                store.set(f"{tag}/reqh/{prev}", enc(ms_prev))   # for the stage before prev: dx hash
        if audit_next:
            store.set(f"{tag}/req/{nxt}", enc(ms_next, key_next))
        ms_req: List[int] = []
        key_req = 0
        if my_auditor is not None:
            k = f"{tag}/req/{self.rank}"
            v = store.get(k)
            ms_req = dec(v)
            key_req = int(v.decode().split(";")[1])
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
        early = self._early_ship
        self._early_ship = None
        sends, recvs = [], []
        if ms_req:
            if early is None:
                sends.append((st.flat.data, my_auditor))
            sends += [(t, my_auditor) for t in x_send]
            sends += [(t, my_auditor) for t in dx_send]
            if keyed:   # answers to the revealed key, after every commitment went out
                sends.append((torch.stack([self._answer_challenge(self.rank, st, m, key_req) for m in ms_req]),
                              my_auditor))
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
        from ..security.grad_audit import K_KEYED
        ans_prev = ans_next = None
        if audit_prev and ms_prev and keyed:
            ans_prev = torch.empty(len(ms_prev), K_KEYED + 4, dtype=torch.float32, device=self.device)
            recvs.append((ans_prev, prev))
        if audit_next and ms_next:
            mir_n = self._audit_mirror(tuple(self.plan.ranges[s + 1]), s + 1)
            if early is None:
                recvs.append((mir_n.flat.data, nxt))
            if keyed:
                ans_next = torch.empty(len(ms_next), K_KEYED + 4, dtype=torch.float32, device=self.device)
                recvs.append((ans_next, nxt))
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
                                                   dx_seen=dx_prev[j] if dx_prev else None,
                                                   answer=None if ans_prev is None else ans_prev[j],
                                                   committed=coms_in.get(prev), key=key_prev))
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
            for j, m in enumerate(ms_next):
                labels = self._audit_targets[m].to(self.device, non_blocking=True)
                res = combine(res, self._audit_one(mir_n, self._audit_outputs.get(m), m, M, labels=labels,
                                                   dx_seen=self._audit_recv_dy.get(m),
                                                   answer=None if ans_next is None else ans_next[j],
                                                   committed=coms_in.get(nxt), key=key_next))
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
