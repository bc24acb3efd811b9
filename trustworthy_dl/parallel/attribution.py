"""Blame attribution and host-side step reports of ``PipelineEngine``: weight integrity, the
per-node (blame, evidence) decision taken identically on every rank from the all-gathered digest,
heartbeat OFFLINE state, and the lagged host report that feeds TrustManager / AttackDetector
mirrors and triggers re-sharding (reference: handle_detected_attack / handle_gradient_attack /
update_trust_scores, distributed_trainer.py:209-322).
"""
from __future__ import annotations

import math
import time
from typing import Dict, List, Optional

import torch

from ..core.trust_manager import NodeStatus, STATUS_CODES
from ..ops import stats as dstats
from ..runtime.commcheck import note_host_sync
from ..security import stage_verifier as SV
from .stage import Stage


class AttributionMixin:
    """Attribution + report processing (mixed into ``PipelineEngine``)."""

    # ================================================================== integrity + attribution
    @torch.no_grad()
    def _integrity_flag(self, st: Stage) -> torch.Tensor:
        """1.0 when the stage's compute weights differ from the checksum taken right after its last
        optimizer step (a write outside the optimizer), else 0.0 — device-side, no sync."""
        cur, st._early_checksum = st._early_checksum, None
        if cur is None:
            cur = dstats.checksum(st.flat.data)
        st._cur_checksum = cur
        # a write between the start of the previous step and its update (during its forward /
        # backward: ADVICE r3) was seen by that step's tail re-check and is reported now
        tail, st._tail_flag = st._tail_flag, None
        ref = st.param_checksum
        if ref is None:  # first step / freshly (re)built or reloaded stage: nothing to compare yet
            st.param_checksum = cur
            return torch.zeros(1, dtype=torch.float32, device=st.device)
        flag = (cur != ref).any().float().reshape(1)
        return flag if tail is None else torch.maximum(flag, tail)

    def _replica_orders(self) -> List[torch.Tensor]:
        key = (self.plan.version, self.dp)
        if self._orders_key != key:
            base = self.replica * self.pp
            self._orders = [torch.tensor([d * self.pp + (r - base) for r in self.plan.ranks], dtype=torch.long,
                                         device=self.device) for d in range(self.dp)]
            self._orders_key = key
        return self._orders

    def _attribute(self, D: torch.Tensor) -> torch.Tensor:
        """Per-node (blame, evidence) for this step, identical on every rank (device, from the
        all-gathered D); ``evidence[n]`` = 1 when n's pipeline replica saw a tampered forward.

        In a pipeline an anomaly echoes: tampered activations of stage s make every later stage's
        output (and, through backward, every stage's gradients) look anomalous too.  Blame goes to
        (a) any stage whose weights failed the integrity check, (b) the EARLIEST stage of each
        pipeline replica with an output anomaly, and (c) gradient anomalies only when the replica
        shows no output / integrity evidence (gradient poisoning does not propagate)."""
        of, gf, pf = D[:, SV.D_OUT_FLAG], D[:, SV.D_GRAD_FLAG], D[:, SV.D_PARAM_FLAG]
        oz = D[:, SV.D_OUT_Z]
        blame = torch.zeros_like(of)
        evidence = torch.zeros_like(of)
        self.t_taint.copy_(torch.maximum(self.t_taint, (pf > 0).float()))
        audited = self._audit_now or self._gsk_on
        akind = torch.zeros_like(of)
        if audited:
            akind, _ = self._audit_vectors(D)
        abad = (akind > 0).float()
        # a tied-weight member applying something else than the sum of the members' contributions
        # (blame), or the tie group's all-reduce fed something else than the committed contributions
        # (evidence: the replica's update is skipped; which member fed it is not identifiable)
        if self._gsk_on:
            gbad, gev = self._tied_mismatch(D)
        else:
            gbad, gev = torch.zeros_like(of), torch.zeros_like(of)
        # proof of tampering (not a statistic): compromises at once (compromise_on_proof)
        self._proof = torch.maximum(torch.maximum((pf > 0).float(), abad), gbad)
        self._proof_kind = akind + gbad * 32.0
        stat_blame = 0.0 if (audited and self.cfg.audit_backward) else 1.0
        for r, idx in enumerate(self._replica_orders()):
            o, g, p = of[idx], gf[idx], pf[idx]
            taint = self.t_taint[idx]
            ev = torch.maximum(o.max(), p.max())
            if audited:
                # deterministic attribution: a tampered forward is blamed only on a recompute
                # mismatch (its own stage, never the downstream echoes) or a failed weight-integrity
                # check; output z-scores do not blame.  Gradient anomalies count only in a replica
                # without such evidence (gradient poisoning does not propagate, tampering does)
                # with the backward audit, gradient z-scores no longer blame either: the
                # deterministic gradient checks (recomputed contribution, applied-vs-committed
                # sketch) do; the statistics still quarantine the update and feed the trust metrics
                a = abad[idx]
                ev = torch.maximum(p.max(), a.max())
                b = torch.maximum(torch.maximum(p, a), g * (1.0 - ev) * stat_blame)
                o = a   # "forward anomaly" below = a recompute mismatch
            elif self.cfg.attribute_flags:
                # earliest anomalous stage; a stage with tampered (integrity-failed, not yet
                # restored) weights counts as anomalous, so the output echoes it causes downstream
                # are neither blamed nor skip the step (its own flag already compromised it)
                if self.cfg.soft_output_z > 0:
                    # a replica with an output flag: softly anomalous earlier stages count too
                    soft = (oz[idx] > self.cfg.soft_output_z).float() * o.max()
                    o = torch.maximum(o, soft)
                a = torch.maximum(o, taint)
                head = (torch.cumsum(a, 0) == 1).float() * a
                first = head * o * (1.0 - taint)
                b = torch.maximum(torch.maximum(p, first), g * (1.0 - ev))
                ev = torch.maximum(p.max(), (head * o * (1.0 - taint)).max())
            else:
                b = torch.maximum(torch.maximum(o, g), p)
            n = idx.numel()
            if self.cfg.global_event_fraction > 0 and n >= 3:
                # pipeline-wide gradient anomaly (every stage's norm jumps together in a loss spike):
                # skip the update, blame nobody, and keep output / gradient blame off for a grace
                # window; integrity (parameter) evidence is never suppressed
                # (with an output anomaly in the replica the gradient flags are echoes of a tampered
                # forward instead, attributed to its earliest stage above)
                glob = (g.sum() >= max(2.0, math.ceil(self.cfg.global_event_fraction * n))).float() * (1.0 - o.max())
                gr = self.t_grace[r:r + 1]
                gr.copy_(torch.maximum(gr - 1.0, torch.zeros_like(gr)) * (1.0 - glob)
                         + glob * float(self.cfg.global_event_grace))
                quiet = torch.maximum(glob, (gr > 0).float())
                if audited:
                    # a recompute mismatch is proof, not a statistic: never quieted (a grace window
                    # opened by an earlier loss spike let tampered steps through in r4's first runs)
                    b = torch.maximum(torch.maximum(p, o), b * (1.0 - quiet))
                    ev = torch.maximum(torch.maximum(p.max(), o.max()), glob)
                else:
                    b = torch.maximum(p, b * (1.0 - quiet))
                    ev = torch.maximum(torch.maximum(p.max(), o.max() * (1.0 - quiet)), glob)
            gb = gbad[idx]
            blame[idx] = torch.maximum(b, gb)
            # a gradient rewritten after the backward skips that stage's update (it does not echo)
            evidence[idx] = torch.maximum(torch.maximum(ev.expand(n), gb), gev[idx])
        return blame, evidence

    # ================================================================== heartbeat -> OFFLINE
    def _apply_offline(self, D: torch.Tensor):
        """A node is OFFLINE while any rank's watchdog reports it silent (union of the all-gathered
        bitmasks, identical on every rank); a node no rank reports any more goes RECOVERING.
        Device-side, so every rank's trust state moves identically without a host sync."""
        N = self.num_nodes
        bits = D[:, SV.D_OFFLINE_MASK].to(torch.int64)
        shifts = torch.arange(N, device=self.device, dtype=torch.int64)
        off = ((bits[:, None] >> shifts[None, :]) & 1).amax(0).to(torch.bool)
        OFF = STATUS_CODES[NodeStatus.OFFLINE]
        was_off = self.t_status == OFF
        self.t_status.copy_(torch.where(off, torch.full_like(self.t_status, OFF),
                                        torch.where(was_off, torch.full_like(self.t_status,
                                                                             STATUS_CODES[NodeStatus.RECOVERING]),
                                                    self.t_status)))

    # ================================================================== host-side report processing
    def flush(self) -> Optional[float]:
        self._consume_reports(upto=None)
        return self.last_loss

    def _consume_reports(self, upto: Optional[int]):
        while self._pending and (upto is None or self._pending[0][0] <= upto):
            step, epoch, host, ev, truth, lasts, mode = self._pending.popleft()
            note_host_sync()
            if ev is not None:
                ev.synchronize()
            self._process_report(step, epoch, host, truth, lasts, mode)

    def _process_report(self, step: int, epoch: int, host: torch.Tensor, truth: Dict[int, bool],
                        loss_ranks: Optional[List[int]] = None, mode=None):
        N = self.num_nodes
        D = host[: N * SV.DIGEST].view(N, SV.DIGEST).tolist()
        values = host[N * SV.DIGEST: N * SV.DIGEST + N].tolist()
        statuses = [int(v) for v in host[N * SV.DIGEST + N:N * SV.DIGEST + 2 * N].tolist()]
        blamed = [v > 0 for v in host[N * SV.DIGEST + 2 * N:N * SV.DIGEST + 3 * N].tolist()]
        audit_kind = [int(v) for v in host[N * SV.DIGEST + 3 * N:N * SV.DIGEST + 4 * N].tolist()]
        audit_bad = [k > 0 for k in audit_kind]
        present = set(self.all_ranks())
        # the loss stages of the plan the step ran under (a re-shard decided by an earlier report
        # may have moved the loss stage since)
        lasts = [n for n in (loss_ranks if loss_ranks is not None else self.last_ranks()) if D[n][SV.D_PRESENT] > 0]
        self.last_loss = sum(D[n][SV.D_LOSS] for n in lasts) / len(lasts) if lasts else None
        detections = []
        for n in range(N):
            row = D[n]
            if n not in present or row[SV.D_PRESENT] <= 0:
                continue
            gt = bool(row[SV.D_ATTACK_TRUTH] > 0)
            out_flag, grad_flag = row[SV.D_OUT_FLAG] > 0, row[SV.D_GRAD_FLAG] > 0
            param_flag = row[SV.D_PARAM_FLAG] > 0
            flagged = blamed[n]
            if flagged:
                kind = self._evidence_kind(param_flag, audit_kind[n], out_flag)
                rec = {"node_id": n, "timestamp": time.time(), "step": step, "attack_type": kind,
                       "output_stats": {"mean": row[SV.D_OUT_MEAN], "std": row[SV.D_OUT_STD],
                                        "z": row[SV.D_OUT_Z]},
                       "gradient_stats": {"norm_l2": row[SV.D_GRAD_L2], "z": row[SV.D_GRAD_Z],
                                          "cosine": row[SV.D_GRAD_COS]},
                       "audit_kind": audit_kind[n], "ground_truth": gt}
                self.attack_history.append(rec)
                self.trust.attack_history[n].append({"timestamp": rec["timestamp"], "step": step,
                                                     "attack_type": kind,
                                                     "previous_trust": self.trust.get_trust_score(n)})
                detections.append(n)
            if self.detector is not None:
                ds = self.detector.detection_stats
                if flagged:
                    ds["total_detections"] += 1
                    k = self._evidence_kind(param_flag, audit_kind[n], out_flag)
                    k = {"output_tampering": "byzantine", "output_anomaly": "byzantine",
                         "gradient_tampering": "byzantine"}.get(k, k)
                    ds["attack_types"][k] = ds["attack_types"].get(k, 0) + 1
                key = ("true_positives" if gt else "false_positives") if flagged else \
                      ("false_negatives" if gt else "true_negatives")
                ds[key] += 1
            if self.attacker is not None and hasattr(self.attacker, "record_detection"):
                self.attacker.record_detection(n, step, flagged, gt)
        metrics = [row[SV.D_METRICS:SV.D_METRICS + 6] for row in D]
        prev_status = {n: self.trust.get_node_status(n) for n in range(N)}
        self.trust.ingest_device_update([values[n] for n in range(N)], [statuses[n] for n in range(N)], metrics,
                                        update_counts=None)
        if detections:
            self.state_flags["under_attack"] = True
        if self.metrics is not None:
            self.metrics.collect_batch_metrics({
                "loss": self.last_loss, "step": step, "epoch": epoch,
                "trust_scores": {i: values[i] for i in range(N)},
                "detections": detections, "grad_norm": [D[n][SV.D_GRAD_L2] for n in range(N)],
                "step_time": self._step_time})
        OFF = STATUS_CODES[NodeStatus.OFFLINE]
        for n in range(N):
            if (statuses[n] == OFF) != (prev_status.get(n) == NodeStatus.OFFLINE):
                self.node_events.append({"node_id": n, "step": step, "timestamp": time.time(),
                                         "event": "offline" if statuses[n] == OFF else "online"})
        self._commit_shadows(step, blamed, statuses)
        newly = [n for n in range(N) if n in present and statuses[n] == STATUS_CODES[NodeStatus.COMPROMISED]
                 and prev_status.get(n) != NodeStatus.COMPROMISED]
        newly += [n for n in range(N) if n in present and statuses[n] == STATUS_CODES[NodeStatus.COMPROMISED]
                  and n not in newly and n in detections]
        if newly and self.cfg.reassign:
            self.reassign(sorted(set(newly)), step)
        elif self.distributed and mode is not None and mode[1] and mode[0] == self.plan.version:
            # weights proven to differ from the auditor's mirror (written outside the verified
            # optimizer) and no re-shard: the stage takes the mirror's verified state back
            heal = [n for n in range(N) if n in present and audit_kind[n] & SV.AK_WHASH]
            if heal:
                self._heal_dist(heal)
        # runtime metrics for the next digest (latency s, utilization, error, uptime)
        util = 1.0 - (self._comm_wait / self._step_time) if self._step_time > 0 else 0.0
        for n in range(N):
            self._host_metrics[n] = [self._comm_wait, max(0.0, min(1.0, util)), 0.0, 1.0]

    def _evidence_kind(self, param_flag: bool, kind: int, out_flag: bool) -> str:
        """Attack record type from the evidence behind a blame (audit bitmask AK_*, 32 = applied
        gradient differs from the committed backward)."""
        if param_flag or kind & SV.AK_WHASH:
            return "model_poisoning"
        if kind & SV.AK_FWD:
            return "output_tampering"
        if kind & (SV.AK_DX | SV.AK_DXHASH):
            return "gradient_tampering"
        if kind & (SV.AK_DW | SV.AK_GAPP):
            return "gradient_poisoning"
        return "output_anomaly" if out_flag and not self.cfg.audit else "gradient_poisoning"
