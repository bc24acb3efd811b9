"""Deterministic recompute audit of ``PipelineEngine``: every stage is audited by the stage that
received its output (the loss stage by its predecessor) on privately chosen micro-batches —
forward output, input gradient and weight-gradient contribution are recomputed on the auditor.
Local mode here; the distributed protocol is in ``audit_dist.py``.

Reference: Byzantine detection by cosine of DIFFERENT stages' outputs (attack_detector.py:143-162),
which over-flags every node.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

from ..security import stage_verifier as SV
from .comm import batched_transfer
from .stage import Stage


class AuditMixin:
    """Recompute audit, local mode + shared helpers (mixed into ``PipelineEngine``)."""

    # ================================================================== deterministic stage cross-check
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

    def _audit_verdict(self, y_seen: torch.Tensor, y_ref: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(mismatch flag, relative max error) of a received output against its recomputation —
        device tensors, no host sync.  Non-finite values count as a mismatch."""
        a, b = y_seen.float(), y_ref.float()
        err = (a - b).abs().amax() / b.abs().amax().clamp_min(1e-12)
        err = torch.nan_to_num(err, nan=1e30, posinf=1e30)
        return (err > self.cfg.audit_tol).float().reshape(1), err.reshape(1)

    def _audit_one(self, st: Stage, x: torch.Tensor, m: int, M: int, y_seen=None, dy=None, labels=None,
                   dx_seen=None, answer=None, committed=None, key: Optional[int] = None, whash=None):
        """All checks of one audited micro-batch ``m`` of stage ``st`` (its own modules in local mode,
        a mirror holding its shipped weights in distributed mode).  Returns device tensors
        (mismatch flag [1], failed-check bitmask [1], worst relative error [1]).

        * forward (AK_FWD): the output the next stage received == f(x; W);
        * input gradient (AK_DX): the gradient sent upstream == the recomputed one for the output
          gradient the audited stage received;
        * weight gradient (AK_DW): the auditee's ``answer`` (CommitmentMixin._answer_challenge) —
          the keyed sketch, under the key revealed only now, of micro-batch m's committed
          contribution — equals the keyed sketch of the recomputed contribution, and the two
          snapshots it was taken from still hash to the ``committed`` values sent before the reveal;
        * weights (AK_WHASH, local mode): the weights in use == the stage's post-update commitment."""
        from ..security.grad_audit import K_KEYED, fold_hash64, keyed_sketch
        bwd = self.cfg.audit_backward and (st.computes_loss or dy is not None)
        y_ref, dx_ref, g_ref = self._recompute(st, x, dy, labels, M, backward=bwd)
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
        if bwd and answer is not None and g_ref is not None and key is not None and committed is not None \
                and 0 <= m < committed.shape[0] - 1:
            segs = self._commit_segments(st)
            ref = keyed_sketch(g_ref, segs, key)
            # scale: the sketch itself, floored at a quarter of the recomputed contribution's norm
            # (a random-sign projection of v has magnitude ~ ||v||): a perturbation of >~ tol x the
            # micro-batch's own gradient fails whatever its direction
            nrm = torch.stack([g_ref[lo:hi].float().square().sum() for lo, hi in segs]).sum().sqrt() \
                if segs else torch.zeros((), device=g_ref.device)
            ans = answer.to(ref.device)
            scale = torch.maximum(ref.abs().amax(), 0.25 * nrm).clamp_min(1e-30)
            e = torch.nan_to_num((ans[:K_KEYED] - ref).abs().amax() / scale, nan=1e30, posinf=1e30).reshape(1)
            hbad = torch.cat([ans[K_KEYED:K_KEYED + 2] != fold_hash64(committed[m]).to(ref.device),
                              ans[K_KEYED + 2:K_KEYED + 4] != fold_hash64(committed[m + 1]).to(ref.device)]).any()
            f = torch.maximum((e > self.cfg.audit_grad_tol).float(), hbad.float().reshape(1))
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
            chosen = [m for m in dict.fromkeys(list(self._audit_ms) + [picks.get(p, -1)])
                      if m >= 0 and "x" in recs.get(m, {})]
            if not chosen or aud not in rows:
                continue
            st = self.stages[p]
            wh = None
            cur, ref = st._cur_checksum, st.param_checksum
            if cur is not None and ref is not None and cur is not ref:
                wh = (fold_hash(cur) != fold_hash(ref)).any().float().reshape(1)
            flag = kind = err = None
            # the key is drawn now, after every commitment of the step was taken (private RNG)
            key = self._mon_rng.getrandbits(64)
            for m in chosen:
                rec = recs[m]
                ans = self._answer_challenge(p, st, m, key) if p in self._gcom else None
                f1, k1, e1 = self._audit_one(st, rec["x"], m, M, y_seen=rec.get("y"),
                                             dy=None if last else rec.get("dy"), labels=rec.get("labels"),
                                             dx_seen=rec.get("dx"), answer=ans, committed=self._gcom.get(p),
                                             key=key, whash=wh)
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
        if not (self.distributed and self._audit_now and self.cfg.audit_prob >= 1.0
                and self._audit_pg is not None):
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
        self._early_ship = (dist.batch_isend_irecv(ops), mirrors)

    def _note_audit_cost(self, host_s: float, ev):
        a = self._audit_cost
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
        a = self._audit_cost
        tl = self._target_log
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
        a = self._audit_cost
        a["bytes"] += sum(t.numel() * t.element_size() for t, _ in list(sends) + list(recvs))
        for ss, rr, g in ((fwd_s, fwd_r, act_g), (bwd_s, bwd_r, grad_g)):
            self._note_peers(ss, rr, "dir" if g is not None else "default")
            batched_transfer(ss, rr, group=g)

    def _audit_mirror(self, rng: Tuple[int, int], sid: int) -> Stage:
        """The audited stage's layers on this GPU (weights overwritten by every audit); one mirror
        per audited layer range (the stage before the loss stage audits two stages)."""
        key = (self.plan.version, tuple(rng))
        cache = self._mirrors
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
