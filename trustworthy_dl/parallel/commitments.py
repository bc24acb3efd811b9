"""Per-micro-batch gradient commitments of ``PipelineEngine`` (security/grad_audit.py).

Commit-then-reveal: after every micro-batch's backward each stage commits the
EXACT hash of its running flat gradient (the tied weight's elements excluded: the tied all-reduce
adds to them) and keeps a snapshot of it; at the step tail it commits the hash of the gradient it is
about to apply.  Only then does its auditor reveal a private per-step key (and which micro-batches
it audits): the stage answers with the keyed full-coverage sketch of the audited micro-batch's
committed contribution (snapshot i+1 - snapshot i, re-hashed against the commitment first), which
the auditor compares with the sketch of its own recomputation (parallel/audit.py).  Every rank
checks applied-hash == last committed hash exactly (``_gsk_mismatch``).

r4 committed sketches under public sign patterns over a public 1/16 sample of the gradient: a
perturbation in the unsampled coordinates or in the null space of the two public sign vectors
passed both checks (attacks/adversarial_attacks.py ``adaptive``, tests/test_keyed_audit.py).  The
public sketch is kept only to rank micro-batches for the targeted audit.

Reference: the gradient check is a host z-score (attack_detector.py:109-141) that cannot see a
sign flip; the phantom ``GradientVerifier`` (distributed_trainer.py:199-205).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch

from ..security import stage_verifier as SV
from .stage import Stage


class CommitmentMixin:
    """Gradient commitments (mixed into ``PipelineEngine``)."""

    # ------------------------------------------------------------------ layout helpers
    def _tied_ids(self, st: Stage) -> List[int]:
        ids = []
        for grp in self.ties:
            for li, attr in grp:
                prm = st.local_param(li, attr)
                if prm is not None:
                    ids.append(id(prm))
        return ids

    def _sketch_for(self, st: Stage):
        """The stage's PUBLIC gradient sketch (security/grad_audit.GradSketch: targeting scores
        only), identical for the stage and any mirror of it (same layer range -> same flat layout,
        signs and tied-weight mask)."""
        from ..security.grad_audit import GradSketch, tied_ranges
        key = (tuple(st.layer_range), st.flat.numel, str(st.device))
        sk = self._gsk_cache.get(key)
        if sk is None:
            a, b = st.layer_range
            sk = self._gsk_cache[key] = GradSketch(st.flat.numel, st.device, seed=self.cfg.seed * 1_000_003 + a * 7919 + b,
                                                   masked=tied_ranges(st.flat, self._tied_ids(st)))
        return sk

    def _commit_segments(self, st: Stage) -> List[Tuple[int, int]]:
        """Flat-gradient ranges the commitments cover: everything but the tied weight's elements
        (the tied all-reduce writes those, possibly while a micro-batch commit is being taken)."""
        from ..security.grad_audit import _segments, tied_ranges
        key = ("seg", tuple(st.layer_range), st.flat.numel)
        segs = self._gsk_cache.get(key)
        if segs is None:
            segs = self._gsk_cache[key] = _segments(st.flat.numel, tied_ranges(st.flat, self._tied_ids(st)))
        return segs

    def _hash_seed(self, st: Stage) -> int:
        a, b = st.layer_range
        return (self.cfg.seed * 1_000_003 + self.global_step * 7919 + a * 31 + b) & 0xFFFFFFFF

    def _snap_buffer(self, node: int, st: Stage, M: int) -> torch.Tensor:
        """[M + 1, numel] fp32 snapshot ring of the stage's running gradient (reused across steps)."""
        key = (node, M, st.flat.numel, str(st.device))
        buf = self._gsnap_cache.get(key)
        if buf is None:
            self._gsnap_cache = {k: v for k, v in self._gsnap_cache.items() if k[0] != node}
            buf = self._gsnap_cache[key] = torch.empty(M + 1, st.flat.numel, dtype=torch.float32, device=st.device)
        return buf

    # ------------------------------------------------------------------ tied weight (public sketch)
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
        key = (prm.numel(), str(st.device))
        sk = self._tsk_cache.get(key)
        if sk is None:
            sk = self._tsk_cache[key] = GradSketch(prm.numel(), st.device, seed=self.cfg.seed * 7 + 424242)
        return sk((prm.main_grad if g is None else g).reshape(-1), sk.offset(self.cfg.seed, self.global_step))

    def _note_tied_pre(self, st: Stage):
        """Right before the tied all-reduce: the stage's own tied-weight gradient contribution."""
        if self._gsk_on:
            t = self._tied_sketch(st)
            if t is not None:
                self._tsk_pre[st.stage_id] = t

    # ------------------------------------------------------------------ per-micro-batch commitments
    def _begin_commitments(self, M: int):
        """Commit state 0 of every local stage (the flat gradient before the first micro-batch's
        backward): its exact hash and snapshot; the public running sketch for targeting."""
        self._gsk_on = bool(self.cfg.audit and self.cfg.audit_backward and self.plan.num_stages > 1 and self.dp == 1)
        self._gsk_run: Dict[int, torch.Tensor] = {}
        self._gcom: Dict[int, torch.Tensor] = {}
        self._gsnap: Dict[int, torch.Tensor] = {}
        self._tsk_pre: Dict[int, torch.Tensor] = {}
        if not self._gsk_on:
            return
        for node, st in self.stages.items():
            self._gcom[node] = torch.zeros(M + 1, dtype=torch.int64, device=st.device)
            self._gsnap[node] = self._snap_buffer(node, st, M)
            self._commit_state(node, st, 0)
            if self._targeted:
                sk = self._sketch_for(st)
                r = torch.zeros(M + 1, 2, dtype=torch.float32, device=st.device)
                r[0].copy_(sk(st.flat.grad, sk.offset(self.cfg.seed, self.global_step)))
                self._gsk_run[node] = r

    def _commit_state(self, node: int, st: Stage, k: int):
        """Commitment k of the running gradient: exact hash + snapshot in one pass."""
        from ..security.grad_audit import word_hash
        word_hash(st.flat.grad, self._commit_segments(st), self._hash_seed(st), snapshot=self._gsnap[node][k],
                  out=self._gcom[node][k:k + 1])

    def _commit_micro(self, node: int, st: Stage, i: int):
        """Micro-batch ``i``'s weight gradients of ``node`` are accumulated: (attack hook, then)
        commit the running gradient."""
        M = len(self._audit_batch)
        if self.attacker is not None and hasattr(self.attacker, "after_micro_backward"):
            if self.attacker.after_micro_backward(node, st.flat.grad, self.global_step, i, M):
                self._truth_now[node] = True
        if node in self._gcom:
            self._commit_state(node, st, i + 1)
        r = self._gsk_run.get(node)
        if r is not None:
            sk = self._sketch_for(st)
            r[i + 1].copy_(sk(st.flat.grad, sk.offset(self.cfg.seed, self.global_step)))

    @torch.no_grad()
    def _answer_challenge(self, node: int, st: Stage, m: int, key: int) -> torch.Tensor:
        """The audited stage's answer for micro-batch ``m`` under the revealed key: [K_KEYED + 4]
        = keyed sketch of snapshot m+1 - snapshot m, then the two snapshots' hashes recomputed NOW
        (each folded to two fp32 halves: the auditor compares them with the commitments it received
        before the reveal, so a snapshot rewritten after committing fails)."""
        from ..security.grad_audit import K_KEYED, fold_hash64, keyed_sketch, word_hash
        segs = self._commit_segments(st)
        snap = self._gsnap[node]
        seed = self._hash_seed(st)
        out = torch.empty(K_KEYED + 4, dtype=torch.float32, device=st.device)
        out[:K_KEYED].copy_(keyed_sketch(snap[m + 1], segs, key, b=snap[m]))
        out[K_KEYED:K_KEYED + 2].copy_(fold_hash64(word_hash(snap[m], segs, seed)))
        out[K_KEYED + 2:K_KEYED + 4].copy_(fold_hash64(word_hash(snap[m + 1], segs, seed)))
        return out

    def _write_commitments(self, node: int, st: Stage, d: torch.Tensor):
        """Digest slots of the gradient commitments: the exact hash of the gradient about to be
        applied (after the tied all-reduce and every hook) and of the committed running gradient
        after the last micro-batch's backward.  They differ when the gradient was rewritten in
        between, on any coordinate."""
        from ..security.grad_audit import fold_hash64, word_hash
        com = self._gcom.get(node) if self._gsk_on else None
        if com is None:
            d[SV.D_GSK_ON:SV.D_GSK_ON + 1].fill_(0.0)
            return
        d[SV.D_GSK_APP:SV.D_GSK_APP + 2].copy_(fold_hash64(word_hash(st.flat.grad, self._commit_segments(st),
                                                                     self._hash_seed(st))))
        d[SV.D_GSK_BWD:SV.D_GSK_BWD + 2].copy_(fold_hash64(com[-1]))
        att = self.attacker
        if att is not None and hasattr(att, "lies_about_commitment") and att.lies_about_commitment(node, self.global_step):
            # simulated liar: its own row claims it committed what it applies
            d[SV.D_GSK_BWD:SV.D_GSK_BWD + 2].copy_(d[SV.D_GSK_APP:SV.D_GSK_APP + 2])
        d[SV.D_GSK_ON:SV.D_GSK_ON + 1].fill_(1.0)
        pre = self._tsk_pre.get(st.stage_id)
        if pre is not None:
            d[SV.D_TSK_PRE:SV.D_TSK_PRE + 2].copy_(pre)
            d[SV.D_TSK_APP:SV.D_TSK_APP + 2].copy_(self._tied_sketch(st))
            d[SV.D_TSK_ON:SV.D_TSK_ON + 1].fill_(1.0)
        else:
            d[SV.D_TSK_ON:SV.D_TSK_ON + 1].fill_(0.0)

    def _gsk_mismatch(self, D: torch.Tensor) -> torch.Tensor:
        """Per-node 1.0 where the applied gradient's hash differs from the committed running
        gradient's (a gradient rewritten after the backward: exact, every coordinate), or (distributed)
        where the last commitment a node reports differs from the one its auditor received.  The
        applied hash itself is the node's own report: a rank that also lies about it is outside what
        this check sees (the recompute audit of its committed contributions still applies)."""
        from ..security.grad_audit import K_SKETCH
        app = D[:, SV.D_GSK_APP:SV.D_GSK_APP + 2]
        com = D[:, SV.D_GSK_BWD:SV.D_GSK_BWD + 2]
        on = (D[:, SV.D_GSK_ON] > 0).float()
        bad = on * (app != com).any(1).float()
        if self.distributed and self.cfg.audit_backward:
            for idx in self._replica_orders():
                S = idx.numel()
                for j in range(S):
                    # the auditor of stage j: stage j + 1, or stage j - 1 for the loss stage
                    if j + 1 < S:
                        rec = D[idx[j + 1], SV.D_GCOM_RECV_PREV:SV.D_GCOM_RECV_PREV + 2]
                    elif j > 0:
                        rec = D[idx[j - 1], SV.D_GCOM_RECV_NEXT:SV.D_GCOM_RECV_NEXT + 2]
                    else:
                        continue
                    n = idx[j]
                    held = (rec > 0).all().float() * on[n]
                    bad[n] = torch.maximum(bad[n], held * (rec - 1.0 != com[n]).any().float())
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
