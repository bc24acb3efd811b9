"""Deterministic recompute audit of ``PipelineEngine``, auditor side: every stage is audited by the
stage that received its output (the loss stage by its predecessor) on privately chosen
micro-batches — forward output, input gradient and weight-gradient contribution recomputed on a
LIVE OPTIMIZER MIRROR of the audited stage — and, every step, its applied gradient and weights are
checked against its commitments (parallel/commitments.py describes the protocol).  Local mode
here; the distributed message flow is in ``audit_dist.py``.

Reference: Byzantine detection by cosine of DIFFERENT stages' outputs (attack_detector.py:143-162),
which over-flags every node; the optimizer step it should guard
(distributed_trainer.py:197-205, :441-446).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist

from ..security import stage_verifier as SV
from .comm import batched_transfer
from .stage import Stage


class AuditMixin:
    """Recompute audit + optimizer mirrors, local mode + shared helpers (mixed into ``PipelineEngine``)."""

    audit_sum_tol = 2e-4    # relative error of sketch(G) vs the sum of the M committed sketches (fp32
    #                         rounding of the ring differences and of the sketch sums: ~1e-6 x M)

    # ================================================================== recompute
    def _recompute(self, st: Stage, x: torch.Tensor, dy: Optional[torch.Tensor] = None,
                   labels: Optional[torch.Tensor] = None, M: int = 1, backward: bool = False):
        """``st``'s forward of one micro-batch as in training (BatchNorm in batch-statistics mode),
        and with ``backward`` its backward from the output gradient ``dy`` (the loss stage: from
        its loss / M, as the schedule runs it), without leaving a trace: module buffers (running
        statistics) are restored and the weight gradients go to a scratch accumulator.  Returns
        (output, input gradient or None, the micro-batch's flat weight gradient or None)."""
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
                dx = xg.grad if xg.is_floating_point() else None
                return y.detach(), dx, scratch
            finally:
                st.flat.set_grad_buffer(saved)
        finally:
            with torch.no_grad():
                for b, v in zip(st.module.buffers(), bufs):
                    b.copy_(v)

    # ================================================================== targeting
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
        drives it toward -1 / 0) and the norm of its public weight-gradient sketch contribution."""
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
            run = self._gsk_run.get(p) if self._gsk_on else None
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
        self._target_log.extend((self.global_step, p, m) for p, m in picks.items())
        return picks

    # ================================================================== optimizer mirrors
    def _audit_mirror(self, rng: Tuple[int, int], sid: int, device=None) -> Stage:
        """The audited stage's layers on this GPU: the auditor's live optimizer mirror of it (its
        own fp32 master + AdamW moments, advanced with the verified gradient every step), or in
        weight-shipping mode a module whose weights every audit overwrites.  One per audited layer
        range and plan (the stage before the loss stage audits two stages)."""
        key = (self.plan.version, tuple(rng))
        cache = self._mirrors
        if key not in cache:
            for k in [k for k in cache if k[0] != self.plan.version]:
                del cache[k]
            # (its gradient-folding hooks stay: the backward audit recomputes weight gradients on it)
            mir = cache[key] = Stage(self.model, rng, sid, self.plan.num_stages, device or self.device, self.dtype,
                                     {"output_detection": False, "gradient_verification": False,
                                      "serialize_streams": True})
            mir.set_clip_exclusions(self._clip_excluded_ids(mir))   # the auditor computes its clip sum
        return cache[key]

    def _clip_excluded_ids(self, st: Stage):
        """Parameters of ``st`` another stage counts in the global clipping norm: members of a tie
        group whose first member lives outside ``st``'s layer range."""
        a, b = st.layer_range
        ex = set()
        for grp in self.ties:
            if a <= grp[0][0] < b:
                continue
            for li, attr in grp:
                prm = st.local_param(li, attr)
                if prm is not None:
                    ex.add(id(prm))
        return ex

    def _clip_sumsq_audited(self, D: torch.Tensor) -> torch.Tensor:
        """Mirror mode: per node, the clipping sum of squares its AUDITOR computed from the gradient
        it shipped (``D_SUMSQ_*`` of the auditor's row), zero where the node's own update is
        quarantined — the global clip scale takes no stage's word for its own gradient norm."""
        sq = torch.zeros(D.shape[0], dtype=torch.float32, device=D.device)
        for idx in self._replica_orders():
            n = idx.numel()
            if n < 2:
                continue
            sq[idx[:-1]] = D[idx[1:], SV.D_SUMSQ_PREV]
            sq[idx[-1:]] = D[idx[-2:-1], SV.D_SUMSQ_NEXT]
        q = torch.maximum((D[:, SV.D_GRAD_FLAG] > 0).float(), (D[:, SV.D_NONFINITE] > 0).float()) \
            if self.cfg.quarantine else torch.zeros_like(sq)
        sq = torch.where((q > 0) | ~torch.isfinite(sq), torch.zeros_like(sq), sq.clamp_min(0.0))
        return sq

    def _invalidate_mirrors(self):
        """Every rank, at the same step: the mirrors' state no longer follows their stages (a step
        they did not see, a checkpoint load); each is re-seeded from its stage before its next use."""
        self._mirror_epoch += 1

    def _mirror_seeded(self, mir: Stage) -> bool:
        return getattr(mir, "_seed_epoch", None) == self._mirror_epoch

    @torch.no_grad()
    def _seed_mirror(self, mir: Stage, master, exp_avg, exp_avg_sq, step: int):
        """Start a mirror from its stage's optimizer state (once per plan / after a load: the one
        point where the auditor takes the auditee's word — the state came from a migration or a
        checkpoint; every update after it is verified)."""
        f = mir.flat
        if master is not None:
            f.master.copy_(master.to(f.device))
            f.exp_avg.copy_(exp_avg.to(f.device))
            f.exp_avg_sq.copy_(exp_avg_sq.to(f.device))
        if f.data is not f.master:
            f.data.copy_(f.master)
        f.step_count = int(step)
        from ..ops.layers import bump_weight_generation
        bump_weight_generation()
        mir._seed_epoch = self._mirror_epoch
        mir._master_root = None
        self._audit_cost["seeds"] += 1

    def _skip_decision(self, D: torch.Tensor, evidence: torch.Tensor, node: int) -> torch.Tensor:
        """[1] 1.0 when ``node``'s update is skipped this step — derived from the all-gathered digest
        only, so the stage and its auditor's mirror take the same decision: its own gradient flag
        or non-finite gradient (quarantine), or tampering evidence in its pipeline replica."""
        z = torch.zeros(1, dtype=torch.float32, device=D.device)
        q = torch.maximum((D[node, SV.D_GRAD_FLAG] > 0).float(), (D[node, SV.D_NONFINITE] > 0).float()).reshape(1) \
            if self.cfg.quarantine else z
        e = evidence[node:node + 1].float() if self.quarantine_on_evidence else z
        return torch.maximum(q, e)

    @torch.no_grad()
    def _mirror_update(self, D: torch.Tensor, evidence: torch.Tensor, total_sumsq: torch.Tensor):
        """Advance every mirror this rank holds with the gradient its stage shipped (verified this
        step) under the clip scale and skip decision every rank derives from the digest."""
        self._mirror_applied = {node: mir for mir, _, node in self._mirror_pending}
        for mir, G, node in self._mirror_pending:
            ctrl = mir.verifier.ctrl
            mir.verifier.set_clip_scale(total_sumsq.to(mir.device), self.cfg.adamw.max_grad_norm)
            ctrl[1:2].copy_(self._skip_decision(D, evidence, node).to(mir.device))
            saved = mir.flat.set_grad_buffer(G)
            try:
                mir.flat.adamw_step(self.cfg.adamw, ctrl=ctrl, zero_grad=False)
            finally:
                mir.flat.set_grad_buffer(saved)
            self._mirror_root_async(mir)
        self._mirror_pending = []

    @torch.no_grad()
    def _heal_from_mirror(self, node: int, st: Stage):
        """Local mirror mode, right after ``node``'s own update: when its auditor proved this step
        that the master weights it committed are not the mirror's (AK_WHASH: a write outside the
        verified optimizer), the stage takes the mirror's verified optimizer state (master, moments,
        compute weights) — device-side, no host read of the verdict: a conditional copy that does
        nothing on a clean step.  The tampering is blamed once and does not outlive the step
        (distributed mode: ``_heal_dist``, from the lagged host report)."""
        mir = self._mirror_applied.get(node)
        if mir is None or self._proof_kind is None:
            return
        flag = ((self._proof_kind[node:node + 1].to(torch.int64) & SV.AK_WHASH) > 0).float()
        f, g = mir.flat, st.flat
        pairs = [(f.master, g.master), (f.exp_avg, g.exp_avg), (f.exp_avg_sq, g.exp_avg_sq)]
        if g.data is not g.master:
            pairs.append((f.data, g.data))
        if st.device.type == "cuda" and all(a.device == b.device for a, b in pairs):
            from ..ops import _lib
            from ..ops._lib import ptr, stream_ptr
            fl = flag.to(st.device)
            for src, dst in pairs:
                _lib.call("tdl_copy_if", ptr(fl), ptr(src), ptr(dst), dst.numel() * dst.element_size(),
                          stream_ptr(st.device))
            return
        if float(flag) > 0:     # CPU tensors (or mirror on another device): a host read
            for src, dst in pairs:
                dst.copy_(src.to(dst.device))
            from ..ops.layers import bump_weight_generation
            bump_weight_generation()

    def _mirror_root_async(self, mir: Stage):
        """Root of the mirror's master weights for the next step's weight check, taken on a side
        stream right after its update (overlaps the next step's forward)."""
        from ..security.grad_audit import merkle_roots
        f = mir.flat
        root = torch.empty(1, 8, dtype=torch.int32, device=f.device)
        if not f.master.is_cuda:
            mir._master_root = merkle_roots(f.master, [(0, f.numel)], out=root)[0]
            return
        key = str(f.device)
        side = self._audit_side.get(key)
        if side is None:
            side = self._audit_side[key] = torch.cuda.Stream(f.device)
        side.wait_stream(torch.cuda.current_stream(f.device))
        with torch.cuda.stream(side):
            merkle_roots(f.master, [(0, f.numel)], out=root)
        mir._master_root = root[0]
        mir._master_root_stream = side

    def _mirror_master_root(self, mir: Stage) -> torch.Tensor:
        from ..security.grad_audit import merkle_root
        r = getattr(mir, "_master_root", None)
        if r is None:
            return merkle_root(mir.flat.master)
        side = getattr(mir, "_master_root_stream", None)
        if side is not None:
            torch.cuda.current_stream(mir.device).wait_stream(side)
        return r

    # ================================================================== checks
    def _audit_verdict(self, y_seen: torch.Tensor, y_ref: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(mismatch flag, relative max error) of a received output against its recomputation —
        device tensors, no host sync.  Non-finite values count as a mismatch."""
        a, b = y_seen.float(), y_ref.float()
        err = (a - b).abs().amax() / b.abs().amax().clamp_min(1e-12)
        err = torch.nan_to_num(err, nan=1e30, posinf=1e30)
        return (err > self.cfg.audit_tol).float().reshape(1), err.reshape(1)

    @staticmethod
    def _seg_rel_err(a: torch.Tensor, ref: torch.Tensor, segs) -> torch.Tensor:
        """max |a - ref| / max |ref| over the segments (device scalar; non-finite -> 1e30)."""
        from ..security.grad_audit import seg_rel_err
        return seg_rel_err(a, ref, segs)

    def _audit_one(self, mir: Stage, x: torch.Tensor, m: int, M: int, y_seen=None, dy=None, labels=None,
                   dx_seen=None, c_m: Optional[torch.Tensor] = None, C: Optional[torch.Tensor] = None,
                   s: Optional[torch.Tensor] = None, key: Optional[int] = None,
                   sT: Optional[torch.Tensor] = None, tkey: Optional[int] = None):
        """Checks of one opened micro-batch ``m``, recomputed on ``mir`` (the live mirror, or the
        stage's own modules / shipped weights outside mirror mode).  Returns device tensors
        (mismatch flag [1], failed-check bitmask [1], worst relative error [1]).

        * forward (AK_FWD): the output the next stage received == f(x; W);
        * input gradient (AK_DX): the gradient sent upstream == the recomputed one for the output
          gradient the audited stage received;
        * contribution (AK_DW): the opened c_m hashes to its commitment, its keyed sketch equals
          the committed s_m bit for bit, and it equals the recomputed contribution; for a tie-group
          member, its tied part's sketch under the shared tie key equals the committed one too."""
        from ..security.grad_audit import keyed_sketch, merkle_root, roots_differ
        bwd = self.cfg.audit_backward and (mir.computes_loss or dy is not None)
        y_ref, dx_ref, g_ref = self._recompute(mir, x, dy, labels, M, backward=bwd)
        z = torch.zeros(1, dtype=torch.float32, device=mir.device)
        kind, err = z.clone(), z.clone()
        if y_seen is not None and not mir.computes_loss:
            f, e = self._audit_verdict(y_seen, y_ref)
            kind += f * SV.AK_FWD
            err = torch.maximum(err, e)
        if bwd and dx_seen is not None and dx_ref is not None:
            f, e = self._audit_verdict(dx_seen, dx_ref)
            kind += f * SV.AK_DX
            err = torch.maximum(err, e)
        if bwd and c_m is not None and g_ref is not None and C is not None and s is not None and 0 <= m < s.shape[0]:
            segs = self._commit_segments(mir)
            c = c_m.to(mir.device)
            hbad = roots_differ(merkle_root(c, segs), C[m])
            sbad = (keyed_sketch(c, self._sum_segments(mir), key) != s[m].to(mir.device)).any().float().reshape(1)
            tr = self._tie_range(mir) if sT is not None else None
            if tr is not None:
                o, nt = tr
                tb = (keyed_sketch(c[o:o + nt], [(0, nt)], tkey) != sT[m].to(mir.device)).any().float().reshape(1)
                sbad = torch.maximum(sbad, tb)
            e = self._seg_rel_err(c, g_ref, segs).reshape(1)
            f = torch.maximum(torch.maximum(hbad, sbad), (e > self.cfg.audit_grad_tol).float())
            kind += f * SV.AK_DW
            err = torch.maximum(err, e)
        return (kind > 0).float(), kind, err

    @torch.no_grad()
    def _verify_applied(self, mir: Stage, C: torch.Tensor, G: torch.Tensor, s: torch.Tensor, key: int):
        """Every step, on data the auditor holds: (AK_GAPP) the shipped gradient hashes to its
        commitment and its keyed sketch equals the sum of the M committed contribution sketches;
        (AK_WHASH) the committed master weights equal this mirror's.  Returns (kind [1], err [1])."""
        from ..security.grad_audit import keyed_sketch, merkle_root, roots_differ
        dev = mir.device
        M = s.shape[0]
        if C.shape[0] != M + 2:
            one = torch.ones(1, device=dev)
            return one * (SV.AK_GAPP + SV.AK_WHASH), one * 1e30
        segs = self._sum_segments(mir)
        G = G.to(dev)
        gbad = roots_differ(merkle_root(G, self._commit_segments(mir)), C[M])
        sg = keyed_sketch(G, segs, key)
        ssum = s.to(dev).float().sum(0)
        from ..security.grad_audit import seg_sumsq
        nrm = seg_sumsq(G, segs).sqrt()
        scale = torch.maximum(sg.abs().amax(), 0.25 * nrm).clamp_min(1e-30)
        e = torch.nan_to_num((sg - ssum).abs().amax() / scale, nan=1e30, posinf=1e30).reshape(1)
        abad = torch.maximum(gbad, (e > self.audit_sum_tol).float())
        wbad = roots_differ(self._mirror_master_root(mir), C[M + 1])
        return abad * SV.AK_GAPP + wbad * SV.AK_WHASH, e

    @torch.no_grad()
    def _write_tie(self, d: torch.Tensor, mir: Stage, G: torch.Tensor, sT: Optional[torch.Tensor],
                   tkey: int, next_slot: bool):
        """Tie-group member audited here: U = sum of its M committed tied contribution sketches,
        G = the sketch of the tied part of the gradient it shipped (= the one its mirror applies),
        N = that part's norm, all under the step's shared tie key, into this auditor's digest row
        (``_tied_mismatch`` compares them across the members).  A malformed ``sT`` leaves ON = 1
        with non-finite U: the member deviates."""
        from ..security.grad_audit import K_KEYED, keyed_sketch
        tr = self._tie_range(mir)
        if tr is None:
            return
        o, nt = tr
        g = G.to(d.device)[o:o + nt]
        bu, bg, bn, bo = (SV.D_TIE_U_NEXT, SV.D_TIE_G_NEXT, SV.D_TIE_N_NEXT, SV.D_TIE_ON_NEXT) if next_slot else \
            (SV.D_TIE_U_PREV, SV.D_TIE_G_PREV, SV.D_TIE_N_PREV, SV.D_TIE_ON_PREV)
        if sT is None or sT.dim() != 2 or sT.shape[1] != K_KEYED:
            d[bu:bu + K_KEYED].fill_(float("nan"))
        else:
            d[bu:bu + K_KEYED].copy_(sT.to(d.device).float().sum(0))
        d[bg:bg + K_KEYED].copy_(keyed_sketch(g, [(0, nt)], tkey))
        d[bn:bn + 1].copy_(torch.linalg.vector_norm(g).reshape(1))
        d[bo:bo + 1].fill_(1.0)

    @staticmethod
    def _combine(acc, res):
        if acc is None:
            return res
        (f0, k0, e0), (f1, k1, e1) = acc, res
        return (torch.maximum(f0, f1), torch.bitwise_or(k0.long(), k1.long()).float(), torch.maximum(e0, e1))

    def _write_verdict(self, d: torch.Tensor, res, next_slot: bool):
        flag, kind, err = res
        base = (SV.D_AUDIT_NEXT, SV.D_AUDITED_NEXT, SV.D_AUDIT_KIND_NEXT) if next_slot else \
            (SV.D_AUDIT_PREV, SV.D_AUDITED_PREV, SV.D_AUDIT_KIND_PREV)
        d[base[0]:base[0] + 1].copy_(flag.to(d.device))
        d[base[1]:base[1] + 1].fill_(1.0)
        d[base[2]:base[2] + 1].copy_(kind.to(d.device))
        d[SV.D_AUDIT_ERR:SV.D_AUDIT_ERR + 1].copy_(torch.maximum(d[SV.D_AUDIT_ERR:SV.D_AUDIT_ERR + 1],
                                                                err.to(d.device)))

    # ================================================================== local protocol
    def _audit(self, rows: Dict[int, torch.Tensor]):
        """Audit of every stage by its auditor (the next stage; the loss stage by its predecessor).

        Mirror mode (backward audit with commitments): every step, commitments -> private key ->
        keyed sketches -> private choice of the opened micro-batches -> opened contributions, all
        through the auditee-side methods of CommitmentMixin (which a lying subclass overrides); the
        auditor checks the applied gradient and the weights every step and recomputes the opened
        micro-batches on its mirror.  Forward-only mode: the opened micro-batches are recomputed on
        the stage's own modules and its weights checked against its post-update checksum.  A verdict
        rides in its auditor's digest row (``D_AUDIT_PREV`` / ``D_AUDIT_NEXT``), so no collective is
        added; a tampered activation or gradient mismatches deterministically, a clean stage
        always matches."""
        if self.distributed:
            self._audit_dist(rows)
            return
        order = list(self.plan.ranks)
        S = len(order)
        M = len(self._audit_batch)
        mirror = self._gsk_on
        picks = self._target_picks(order) if self._targeted else {}
        coms: Dict[int, Tuple[torch.Tensor, torch.Tensor]] = {}
        tkey = None
        if mirror:
            # every audited stage commits before any key exists (the tie key is shared by the tie
            # group's members: drawn after all of them committed)
            for k in range(S):
                if k == S - 1 and not self.cfg.audit_backward:
                    continue
                aud = order[k + 1] if k < S - 1 else order[k - 1]
                if aud in rows:
                    p = order[k]
                    dev = self.stages[aud].device
                    coms[p] = (self._contrib_commitments(p, self.stages[p]).to(dev),
                               self._applied_gradient(p, self.stages[p]).to(dev))
            if self._tie_members():
                tkey = self._mon_rng.getrandbits(63)
        for k in range(S):
            p = order[k]
            last = k == S - 1
            if last and not self.cfg.audit_backward:
                continue
            aud = order[k + 1] if not last else order[k - 1]
            if aud not in rows:
                continue
            st = self.stages[p]
            recs = self._audit_rec.get(p, {})
            chosen = [m for m in dict.fromkeys(list(self._audit_ms) + [picks.get(p, -1)])
                      if m >= 0 and "x" in recs.get(m, {})] if self._audit_now else []
            res = None
            C = s = key = sT = None
            opened: List[torch.Tensor] = []
            if mirror:
                dev = self.stages[aud].device
                mir = self._audit_mirror(st.layer_range, st.stage_id, dev)
                if not self._mirror_seeded(mir):
                    self._seed_mirror(mir, *self._optimizer_state(p, st))
                # the key is drawn only after the commitments exist, the opened set only after the
                # sketches (private RNG; a lying auditee-side method sees them in that order)
                C, G = coms[p]
                key = self._mon_rng.getrandbits(63)
                s = self._contrib_sketches(p, st, key).to(dev)
                if tkey is not None and self._tie_range(st) is not None:
                    sT = self._tie_sketches(p, st, tkey)
                    sT = sT.to(dev) if sT is not None else None
                    self._write_tie(rows[aud], mir, G, sT, tkey, next_slot=last)
                opened = self._open_contributions(p, st, chosen)
                kd, e = self._verify_applied(mir, C, G, s, key)
                res = ((kd > 0).float(), kd, e)
                self._mirror_pending.append((mir, G, p))
                rows[aud][SV.D_MIRROR:SV.D_MIRROR + 1].fill_(1.0)
                slot = SV.D_SUMSQ_NEXT if last else SV.D_SUMSQ_PREV
                rows[aud][slot:slot + 1].copy_(mir.clip_sumsq(G).reshape(1).to(rows[aud].device))
            else:
                if not chosen:
                    continue
                mir = st
                cur, ref = st._cur_checksum, st.param_checksum
                if cur is not None and ref is not None and cur is not ref:
                    wh = (cur != ref).any().float().reshape(1)
                    res = ((wh > 0).float(), wh * SV.AK_WHASH, torch.zeros(1, device=st.device))
            for j, m in enumerate(chosen):
                rec = recs[m]
                res = self._combine(res, self._audit_one(
                    mir, rec["x"].to(mir.device), m, M, y_seen=rec.get("y"), dy=None if last else rec.get("dy"),
                    labels=rec.get("labels"), dx_seen=rec.get("dx"), c_m=opened[j] if opened else None,
                    C=C, s=s, key=key, sT=sT, tkey=tkey))
            if res is not None:
                self._write_verdict(rows[aud], res, next_slot=last)

    # ================================================================== weight shipping (no mirror)
    def _audit_early_ship(self, st: Stage):
        """Distributed audit without optimizer mirrors (data-parallel replicas, or the forward-only
        audit), weights part: posted BEFORE the 1F1B schedule on the audit communicator so the
        transfer overlaps the step.  The weights sent are those of the step (posted after the
        attacker's parameter hook, nothing writes them before the optimizer, which runs after the
        audit waited for the transfer); shipping every step reveals nothing about the private
        choice, so this runs only when every step is audited (``audit_prob`` = 1).  In mirror mode
        nothing is shipped: the auditor holds its own verified copy."""
        self._early_ship = None
        if not (self.distributed and self._audit_now and self.cfg.audit_prob >= 1.0
                and self._audit_pg is not None) or self._gsk_on:
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
        a = self._audit_cost
        a["bytes"] += sum(t.numel() * t.element_size() for t, _ in sends + recvs)
        a["sent"] += sum(t.numel() * t.element_size() for t, _ in sends)
        self._early_ship = (dist.batch_isend_irecv(ops), mirrors)

    # ================================================================== accounting
    def _note_audit_cost(self, host_s: float, ev):
        a = self._audit_cost
        a["steps"] += 1
        a["host_s"] += host_s
        if ev is not None:
            a["events"].append(ev)
            if len(a["events"]) > 512:
                del a["events"][:256]

    def audit_summary(self) -> Dict[str, float]:
        """Per-step cost of the audit protocol on this rank (call after a device sync): P2P bytes
        it sent + received and sent alone per step (applied gradient, opened contributions, inputs,
        input gradients), without the one-off mirror seeds (``seed_bytes`` received in total), host
        wall time of the audit phase, device time between its first and last kernel (HIP events),
        device memory it holds (contribution rings + mirrors)."""
        a = self._audit_cost
        tl = self._target_log
        if not a or not a["steps"]:
            return {"steps": 0, "targeted_extra": len(tl)}
        gpu = [e0.elapsed_time(e1) for e0, e1 in a["events"] if e1.query()]
        return {"steps": a["steps"], "bytes_per_step": a["bytes"] / a["steps"],
                "sent_bytes_per_step": a["sent"] / a["steps"],
                "seed_bytes": a["seed_bytes"], "mirror_seeds": a["seeds"],
                "host_ms_per_step": 1e3 * a["host_s"] / a["steps"],
                "device_ms_per_step": (sum(gpu) / len(gpu)) if gpu else None,
                "memory_bytes": self.audit_memory_bytes(), "targeted_extra": len(tl), "heals": a.get("heals", 0)}

    def _audit_transfer(self, sends, recvs, prev, nxt, act_g, grad_g):
        """Audit traffic: toward the next stage on the activation communicator, toward the
        previous one on the gradient communicator (async P2P mode; grouped mode: default group),
        as two batched exchanges in the same order on every rank."""
        fwd_s = [(t, r) for t, r in sends if r == nxt]
        fwd_r = [(t, r) for t, r in recvs if r == prev]
        bwd_s = [(t, r) for t, r in sends if r == prev]
        bwd_r = [(t, r) for t, r in recvs if r == nxt]
        a = self._audit_cost
        a["bytes"] += sum(t.numel() * t.element_size() for t, _ in list(sends) + list(recvs))
        a["sent"] += sum(t.numel() * t.element_size() for t, _ in sends)
        for ss, rr, g in ((fwd_s, fwd_r, act_g), (bwd_s, bwd_r, grad_g)):
            self._note_peers(ss, rr, "dir" if g is not None else "default")
            batched_transfer(ss, rr, group=g)

    def _audit_vectors(self, D: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Per-node (failed-check bitmask, audited) from the digest, identical on every rank: a
        stage's verdict sits in the row of its auditor (the next stage of its pipeline replica; the
        loss stage's in its predecessor's ``*_NEXT`` slots), plus the cross-party hash checks, each
        comparing what two OTHER ranks hold: the input gradients a stage shipped to its auditor vs
        those its upstream stage received, its shipped inputs vs the outputs its upstream stage
        sent, and (weight-shipping mode) the weights its auditor received vs its post-update
        commitment."""
        R = 8
        N = D.shape[0]
        kind = torch.zeros(N, dtype=torch.float32, device=D.device)
        done = torch.zeros_like(kind)
        bwd = self.cfg.audit_backward

        def differ(a, b):
            both = ((a[..., 0] >= 0) & (b[..., 0] >= 0)).float()
            return both * (a != b).any(-1).float()
        for idx in self._replica_orders():
            n = idx.numel()
            if n < 2:
                continue
            a, p = idx[1:], idx[:-1]
            kind[p] = D[a, SV.D_AUDIT_KIND_PREV] + (D[a, SV.D_AUDIT_PREV] > 0).float() * \
                (D[a, SV.D_AUDIT_KIND_PREV] <= 0).float() * SV.AK_FWD
            done[p] = D[a, SV.D_AUDITED_PREV]
            if self.distributed:
                kind[p] += differ(D[p, SV.D_WHASH:SV.D_WHASH + R], D[a, SV.D_WHASH_PREV:SV.D_WHASH_PREV + R]) \
                    * SV.AK_WHASH
                if n >= 3:
                    # stage j (1 <= j <= n-2) shipped its x / dx to idx[j+1]; idx[j-1] sent / received them
                    q, up, au = idx[1:-1], idx[:-2], idx[2:]
                    bad = torch.maximum(
                        differ(D[up, SV.D_DXHASH_RECV:SV.D_DXHASH_RECV + R], D[au, SV.D_DXHASH_SHIP:SV.D_DXHASH_SHIP + R]),
                        differ(D[up, SV.D_XHASH_SENT:SV.D_XHASH_SENT + R], D[au, SV.D_XHASH_SHIP:SV.D_XHASH_SHIP + R]))
                    kind[q] += bad * SV.AK_DXHASH
            if bwd:
                # 1-element index tensors: a 0-d device tensor as an index is read back to the host
                L, A = idx[-1:], idx[-2:-1]
                kind[L] = D[A, SV.D_AUDIT_KIND_NEXT]
                done[L] = D[A, SV.D_AUDITED_NEXT]
                if self.distributed:
                    kind[L] += differ(D[L, SV.D_WHASH:SV.D_WHASH + R], D[A, SV.D_WHASH_NEXT:SV.D_WHASH_NEXT + R]) \
                        * SV.AK_WHASH
        return kind, done
