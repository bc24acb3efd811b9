"""Auditee side of the gradient protocol of ``PipelineEngine`` (security/grad_audit.py; the
auditor side is parallel/audit.py and audit_dist.py).

Per step, every audited stage A (its auditor V: the next stage, or the previous one for the loss
stage):

1. during the backward, after micro-batch i's weight gradients: c_i = g - prev, prev = g into a
   ring of M contributions (the tied weight's part of the last one is taken right before the tied
   all-reduce when that starts early; the all-reduce adds the other member's contributions to the
   tied rows of G, so the sum check of step 5 leaves them out and the members' auditors check them
   against each other instead, step 6);
2. **commit**: A sends V the BLAKE2s Merkle roots of c_0..c_{M-1}, of the gradient G it applies and
   of its fp32 master weights (``_contrib_commitments``), and ships G itself;
3. **key**: only after V RECEIVED the commitments does it reveal a private sketch key; A answers
   with the keyed sketches s_i of all M contributions (``_contrib_sketches``);
4. **open**: only after V received the sketches does it reveal which k micro-batches it audits; A
   ships those c_m (``_open_contributions``);
5. V checks with data it hashes itself: root(c_m) == commitment, sketch(c_m) == s_m (bit exact),
   c_m == V's recomputation of micro-batch m; root(G) == commitment, sketch(G) == sum_i s_i; the
   committed master == V's LIVE OPTIMIZER MIRROR of A (fp32 master + AdamW moments, advanced every
   step with the verified G under the clip scale / quarantine decision every rank derives from the
   all-gathered digest).  So A cannot apply anything but sum_i c_i (a lie in any s_i or c_i is
   opened with probability >= k/M per step), cannot apply something else than the G it shipped
   (the mirror diverges: caught at the next step's weight check), and cannot rewrite its weights
   outside the optimizer.
6. **tie**: for the tied embedding / LM-head weight, each member's auditor adds a private part to a
   shared tie key after reading its auditee's commitments; each member answers with the keyed
   sketches of its M contributions' tied rows under that key (opened ones verified like s_m), and
   its auditor publishes U = their sum and sketch(tied rows of G).  Every rank checks that each
   member applies U_embedding + U_head (``_tied_mismatch``).

Every auditee-side answer is a method a lying rank can override (tests/test_lying_rank.py runs
such subclasses as gloo ranks); no check trusts a value the audited rank reports about itself.

Reference: the gradient check is a host z-score (attack_detector.py:109-141) that cannot see a
sign flip; the phantom ``GradientVerifier`` (distributed_trainer.py:199-205); the optimizer step
that should only apply verified gradients (distributed_trainer.py:197-205, :441-446).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch

from ..security import stage_verifier as SV
from .stage import Stage


class CommitmentMixin:
    """Gradient commitments, auditee side (mixed into ``PipelineEngine``)."""

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
        """Flat ranges the Merkle commitments and the recompute comparison cover: all of it (the
        tied weight's own per-micro-batch contributions included)."""
        return [(0, st.flat.numel)]

    def _sum_segments(self, st: Stage) -> List[Tuple[int, int]]:
        """Flat ranges of the keyed sum check sketch(G) = sum_i s_i: everything but the tied
        weight's elements (its applied gradient is the tie group's all-reduce of the members'
        contributions, checked across the members' auditors: ``_tied_mismatch``)."""
        from ..security.grad_audit import _segments, tied_ranges
        key = ("seg", tuple(st.layer_range), st.flat.numel)
        segs = self._gsk_cache.get(key)
        if segs is None:
            segs = self._gsk_cache[key] = _segments(st.flat.numel, tied_ranges(st.flat, self._tied_ids(st)))
        return segs

    def _ring_buffers(self, node: int, st: Stage, M: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """([M, numel] contribution ring, [numel] previous running gradient), fp32, reused across
        steps: (M + 1) x the stage's gradient memory (``audit_memory_bytes``)."""
        key = (node, M, st.flat.numel, str(st.device))
        buf = self._gring_cache.get(key)
        if buf is None:
            self._gring_cache = {k: v for k, v in self._gring_cache.items() if k[0] != node}
            buf = self._gring_cache[key] = (torch.empty(M, st.flat.numel, dtype=torch.float32, device=st.device),
                                            torch.empty(st.flat.numel, dtype=torch.float32, device=st.device))
        return buf

    def audit_memory_bytes(self) -> int:
        """Device bytes the protocol holds on this rank: contribution rings + optimizer mirrors."""
        n = sum(r.numel() * 4 + p.numel() * 4 for r, p in self._gring_cache.values())
        for mir in self._mirrors.values():
            f = mir.flat
            n += sum(t.numel() * t.element_size() for t in {id(t): t for t in (f.master, f.data, f.exp_avg,
                                                                             f.exp_avg_sq, f.grad)}.values())
            g_in = getattr(mir, "_g_in", None)
            if g_in is not None:
                n += g_in.numel() * 4
        return n

    # ------------------------------------------------------------------ tied weight
    def _tie_members(self) -> List[int]:
        """Stage positions (in the replica's order) holding a member of the first tie group, when
        the group spans more than one stage (GPT-2: the embedding stage and the LM-head stage)."""
        if not self.ties:
            return []
        pos = sorted({i for li, _ in self.ties[0] for i, (a, b) in enumerate(self.plan.ranges) if a <= li < b})
        return pos if len(pos) > 1 else []

    @staticmethod
    def _tie_key_of(parts) -> int:
        """The step's shared tie key from every member auditor's private contribution (each posted
        only after its auditee's commitments were read): no member knows it before committing."""
        import hashlib
        h = hashlib.blake2b(",".join(str(int(v)) for v in sorted(parts)).encode(), digest_size=8).digest()
        return int.from_bytes(h, "little") & ((1 << 63) - 1)

    def _tie_range(self, st: Stage) -> Optional[Tuple[int, int]]:
        """(offset, numel) of this stage's member of a cross-stage tie group in its flat buffer."""
        if st.stage_id not in self._tie_members():
            return None
        for li, attr in self.ties[0]:
            prm = st.local_param(li, attr)
            if prm is not None:
                for q, o, n in zip(st.flat.params, st.flat.offsets, st.flat.sizes):
                    if q is prm:
                        return o, n
        return None

    def _node_of(self, st: Stage) -> int:
        for n, s_ in self.stages.items():
            if s_ is st:
                return n
        return -1

    def _note_tied_pre(self, st: Stage):
        """Right before a tied all-reduce: when it is launched before the last micro-batch's
        contribution was taken (the early path, from an autograd hook), take the tied weight's part
        of that contribution now — the all-reduce rewrites those elements in place."""
        node = self._node_of(st)
        ring = self._gring.get(node) if self._gsk_on else None
        tr = self._tie_range(st)
        if ring is None or tr is None or self._gcount.get(node, 0) != ring.shape[0] - 1:
            return
        from ..security.grad_audit import contrib_snap
        o, n = tr
        contrib_snap(st.flat.grad[o:o + n], self._gprev[node][o:o + n], ring[-1][o:o + n])
        self._tied_snapped[node] = True

    # ------------------------------------------------------------------ per-micro-batch contributions
    def _begin_commitments(self, M: int):
        """Open the step's contribution rings (prev := the running gradient before the first
        micro-batch's backward) and, for the targeted audit, the public running sketches."""
        self._gsk_on = bool(self.cfg.audit and self.cfg.audit_backward and self.plan.num_stages > 1 and self.dp == 1)
        self._gring: Dict[int, torch.Tensor] = {}
        self._gprev: Dict[int, torch.Tensor] = {}
        self._gcom: Dict[int, torch.Tensor] = {}
        self._gcount: Dict[int, int] = {}
        self._tied_snapped: Dict[int, bool] = {}
        self._gsk_run: Dict[int, torch.Tensor] = {}
        self._mirror_pending = []
        self._mirror_applied = {}
        if not self._gsk_on:
            # a step whose gradients no mirror sees: every mirror must be re-seeded before it is used
            self._invalidate_mirrors()
            return
        for node, st in self.stages.items():
            ring, prev = self._ring_buffers(node, st, M)
            prev.copy_(st.flat.grad)
            self._gring[node], self._gprev[node] = ring, prev
            # [M + 2, 8] roots: filled as the step goes (contributions, master), the applied gradient last
            self._gcom[node] = torch.empty(M + 2, 8, dtype=torch.int32, device=st.device)
            if self._targeted:
                sk = self._sketch_for(st)
                r = torch.zeros(M + 1, 2, dtype=torch.float32, device=st.device)
                r[0].copy_(sk(st.flat.grad, sk.offset(self.cfg.seed, self.global_step)))
                self._gsk_run[node] = r

    def _commit_micro(self, node: int, st: Stage, i: int):
        """Micro-batch ``i``'s weight gradients of ``node`` are accumulated: (attack hook, then)
        its contribution into the ring."""
        from ..security.grad_audit import contrib_snap
        M = len(self._audit_batch)
        if self.attacker is not None and hasattr(self.attacker, "after_micro_backward"):
            if self.attacker.after_micro_backward(node, st.flat.grad, self.global_step, i, M):
                self._truth_now[node] = True
        ring = self._gring.get(node)
        if ring is not None:
            self._gcount[node] = i + 1
            if self._tied_snapped.get(node) and i == ring.shape[0] - 1:
                g, prev = st.flat.grad, self._gprev[node]
                for lo, hi in self._sum_segments(st):   # the tied part was taken before its all-reduce
                    contrib_snap(g[lo:hi], prev[lo:hi], ring[i][lo:hi])
            else:
                contrib_snap(st.flat.grad, self._gprev[node], ring[i])
            # its commitment on the verifier's side stream (two launches: leaves + level 1, the rest
            # of the tree), overlapping the next micro-batches' compute instead of the step's tail
            self._on_side(st, lambda: self._root_into(ring[i], self._commit_segments(st), self._gcom[node][i:i + 1]))
        r = self._gsk_run.get(node)
        if r is not None:
            sk = self._sketch_for(st)
            r[i + 1].copy_(sk(st.flat.grad, sk.offset(self.cfg.seed, self.global_step)))

    def _commit_master(self, node: int, st: Stage):
        """The root of the master weights this step runs with (taken once its weights are final for
        the step, ScheduleMixin._attack_params), on the side stream, overlapped with the forward."""
        com = self._gcom.get(node) if self._gsk_on else None
        if com is not None:
            M = com.shape[0] - 2
            self._on_side(st, lambda: self._root_into(st.flat.master, [(0, st.flat.numel)], com[M + 1:M + 2]))

    @staticmethod
    def _root_into(x: torch.Tensor, segs, out: torch.Tensor):
        from ..security.grad_audit import merkle_roots
        merkle_roots(x, segs, out=out)

    @staticmethod
    def _roots_into(x: torch.Tensor, segs, batch: int, stride: int, out: torch.Tensor):
        from ..security.grad_audit import merkle_roots
        merkle_roots(x, segs, batch=batch, stride=stride, out=out)

    @staticmethod
    def _on_side(st: Stage, fn):
        """Run ``fn`` (device work reading tensors the compute stream has written) on the stage's
        verification side stream after the compute stream's work so far; CPU / serialized: inline."""
        side = getattr(st.verifier, "side", None)
        if side is None or not st.flat.grad.is_cuda:
            fn()
            return
        cur = torch.cuda.current_stream(st.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            fn()

    def _join_side(self, st: Stage):
        side = getattr(st.verifier, "side", None)
        if side is not None and st.flat.grad.is_cuda:
            torch.cuda.current_stream(st.device).wait_stream(side)

    # ------------------------------------------------------------------ auditee answers (overridable)
    def _applied_gradient(self, node: int, st: Stage) -> torch.Tensor:
        """The flat gradient this stage applies (and ships to its auditor's mirror)."""
        return st.flat.grad

    @torch.no_grad()
    def _contrib_commitments(self, node: int, st: Stage) -> torch.Tensor:
        """[M + 2, 8] int32 roots: the M contributions, the applied gradient, the fp32 master
        weights (before this step's update = after the previous one)."""
        from ..security.grad_audit import merkle_root
        self._join_side(st)      # the contributions' and the master's roots were taken on the side stream
        C = self._gcom[node].clone()
        M = C.shape[0] - 2
        C[M].copy_(merkle_root(self._applied_gradient(node, st), self._commit_segments(st)))
        return C

    @torch.no_grad()
    def _contrib_sketches(self, node: int, st: Stage, key: int) -> torch.Tensor:
        """[M, K_KEYED] keyed sketches of the M committed contributions under the revealed key
        (the tied weight's elements excluded: ``_tie_sketches``)."""
        from ..security.grad_audit import keyed_sketch
        ring = self._gring[node]
        M, n = ring.shape
        return keyed_sketch(ring, self._sum_segments(st), key, batch=M, stride=n)

    @torch.no_grad()
    def _tie_sketches(self, node: int, st: Stage, tie_key: int) -> Optional[torch.Tensor]:
        """[M, K_KEYED] keyed sketches of the tied weight's part of the M contributions under the
        step's shared tie key, indexed parameter-locally (so every member's sketches add up)."""
        from ..security.grad_audit import keyed_sketch
        tr = self._tie_range(st)
        if tr is None:
            return None
        o, nt = tr
        ring = self._gring[node]
        M, n = ring.shape
        return keyed_sketch(ring.reshape(-1)[o:], [(0, nt)], tie_key, batch=M, stride=n)

    def _open_contributions(self, node: int, st: Stage, ms: List[int]) -> List[torch.Tensor]:
        """The contributions of the opened micro-batches (views into the ring)."""
        ring = self._gring[node]
        return [ring[m] for m in ms]

    def _optimizer_state(self, node: int, st: Stage) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor, int]:
        """(master, exp_avg, exp_avg_sq, step count): seeds the auditor's mirror once per plan."""
        f = st.flat
        return f.master, f.exp_avg, f.exp_avg_sq, f.step_count

    # ------------------------------------------------------------------ digest slots + tied check
    def _write_commitments(self, node: int, st: Stage, d: torch.Tensor):
        """Hook point for the stage's own digest row before the audit (the checks themselves are
        all computed by auditors; a lying subclass overrides this to misreport its statistics)."""
        return

    def _tied_mismatch(self, D: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Per node (blame, evidence) of the tied-weight check, identical on every rank, from values
        the tie members' AUDITORS computed: U_X = sum of member X's committed tied contribution
        sketches (each opened one verified against X's commitment and recompute), G_X = sketch of the
        tied gradient X shipped (and its mirror applies), under the step's shared tie key.  Every
        member must apply sum_X U_X.  A member whose G deviates while another's matches applied
        something else: blamed.  When every member deviates alike, the all-reduce was fed something
        other than the committed contributions — which member did it is not identifiable from the
        sum — so the replica's update is skipped (evidence) and nobody is blamed."""
        from ..security.grad_audit import K_KEYED
        N = D.shape[0]
        bad = torch.zeros(N, dtype=torch.float32, device=D.device)
        ev = torch.zeros_like(bad)
        mem = self._tie_members()
        if not mem:
            return bad, ev
        K = K_KEYED
        for idx in self._replica_orders():
            S = idx.numel()
            if S < 2 or max(mem) >= S:
                continue
            us, gs, ns, ons, nodes = [], [], [], [], []
            for j in mem:
                if j + 1 < S:
                    a, base = idx[j + 1:j + 2], (SV.D_TIE_U_PREV, SV.D_TIE_G_PREV, SV.D_TIE_N_PREV, SV.D_TIE_ON_PREV)
                else:
                    a, base = idx[j - 1:j], (SV.D_TIE_U_NEXT, SV.D_TIE_G_NEXT, SV.D_TIE_N_NEXT, SV.D_TIE_ON_NEXT)
                us.append(D[a, base[0]:base[0] + K].reshape(K))
                gs.append(D[a, base[1]:base[1] + K].reshape(K))
                ns.append(D[a, base[2]].reshape(()))
                ons.append((D[a, base[3]] > 0).float().reshape(()))
                nodes.append(idx[j:j + 1])
            on = torch.stack(ons).amin()
            tot = torch.stack(us).sum(0)
            dev = []
            for g, n_ in zip(gs, ns):
                sc = torch.maximum(torch.maximum(tot.abs().amax(), g.abs().amax()), 0.25 * n_).clamp_min(1e-30)
                e = torch.nan_to_num((g - tot).abs().amax() / sc, nan=1e30, posinf=1e30)
                dev.append((e > self.audit_sum_tol).float() * on)
            dev = torch.stack(dev)
            every = dev.amin()
            for d_, nd in zip(dev, nodes):
                bad[nd] = torch.maximum(bad[nd], (d_ * (1.0 - every)).reshape(1))
                ev[nd] = torch.maximum(ev[nd], (d_ * every).reshape(1))
            if every.numel():
                ev[idx] = torch.maximum(ev[idx], every.expand(S))
        return bad, ev
