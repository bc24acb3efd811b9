"""Data parallelism over pipeline replicas for ``PipelineEngine``: Byzantine-robust gradient mean,
cross-replica direction check and weight-digest audit (reference: the imported-but-unused DDP,
distributed_trainer.py:9, and "Gradient Agg.", README.md:31).
"""
from __future__ import annotations

import logging
import time
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..core.trust_manager import NodeStatus, STATUS_CODES
from ..runtime.commcheck import note_host_sync
from ..security import stage_verifier as SV
from .comm import all_gather_rows
from .stage import Stage

logger = logging.getLogger(__name__)


class DataParallelMixin:
    """Pipeline-replica data parallelism (mixed into ``PipelineEngine``)."""

    # ================================================================== data parallelism (pipeline replicas)
    def all_ranks(self) -> List[int]:
        """Every rank holding a stage: the plan's ranks in each replica."""
        if self.dp == 1:
            return list(self.plan.ranks)
        base = self.replica * self.pp
        return [d * self.pp + (r - base) for d in range(self.dp) for r in self.plan.ranks]

    def last_ranks(self) -> List[int]:
        base = self.replica * self.pp
        return [d * self.pp + (self.plan.ranks[-1] - base) for d in range(self.dp)]

    def _dp_group_ranks(self) -> List[int]:
        pos = self.rank % self.pp
        return [d * self.pp + pos for d in range(self.dp)]

    def _dp_aggregate(self, D: torch.Tensor, evidence: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Byzantine-robust gradient mean across this stage's replicas, all on device.

        A replica is left out when its own verifier flagged the gradient, it produced non-finite
        values, its node is COMPROMISED, or (>= 3 replicas) its gradient norm is an outlier
        against the replicas' median.  Each rank scales its flat gradient by ok / n_ok and the
        replicas all-reduce (sum) -> mean of the trusted replicas; if none is trusted the step is
        skipped on every replica (weights stay identical).  Returns the global sum of squares of the
        aggregated gradient (for clipping), from one extra scalar all-reduce."""
        st = self.my_stage()
        ranks = self._dp_group_ranks()
        idx = self._index_tensor(ranks)
        rows = D[idx]
        bad = torch.maximum(rows[:, SV.D_GRAD_FLAG], (rows[:, SV.D_NONFINITE] > 0).float())
        bad = torch.maximum(bad, (self.t_status[idx] == STATUS_CODES[NodeStatus.COMPROMISED]).float())
        if evidence is not None:
            bad = torch.maximum(bad, evidence[idx])  # the replica's forward was tampered
        if len(ranks) >= 3:
            norms = rows[:, SV.D_GRAD_L2]
            med = norms.median()
            ratio = norms / torch.clamp(med, min=1e-30)
            tau = float(self.cfg.outlier_ratio)
            bad = torch.maximum(bad, ((ratio > tau) | (ratio < 1.0 / tau)).float())
            if st is not None and self.cfg.robust_aggregation:
                bad = torch.maximum(bad, self._dp_direction_outliers(st, len(ranks), bad[ranks.index(self.rank)]))
        if not self.cfg.robust_aggregation:
            bad = torch.zeros_like(bad)
        ok = 1.0 - bad
        n_ok = ok.sum()
        me = ranks.index(self.rank)
        w = ok[me] / torch.clamp(n_ok, min=1.0)
        if st is not None:
            st.flat.grad.mul_(w)
            # an excluded replica contributes exactly zero: NaN/Inf * 0 is NaN, so clear it outright
            st.flat.grad.masked_fill_(w <= 0, 0.0)
            dist.all_reduce(st.flat.grad, group=self.dp_group)
            st.verifier.ctrl[1:2].copy_((n_ok < 0.5).float().reshape(1))
            sq = st.clip_sumsq(st.flat.grad).reshape(1)
        else:
            sq = torch.zeros(1, device=self.device)
        self._dp_excluded = bad
        dist.all_reduce(sq)
        return (sq / self.dp).reshape(())

    def _dp_direction_outliers(self, st: Stage, n: int, bad_me: torch.Tensor) -> torch.Tensor:
        """Cross-replica direction check (the reference's ``detect_byzantine_behavior`` Gram-matrix
        idea, attack_detector.py:143-162, on a sketch): every replica takes the same strided 1/64
        sample of its flat gradient, one small all-reduce sums the unit-normalised samples of the
        replicas not already excluded, and each replica's cosine to the SUM OF THE OTHERS is
        all-gathered.  A replica pointing against its peers (a sign
        flip, which no per-replica statistic sees) is an outlier: cosine < 0 and more than
        ``direction_margin`` below the replicas' median.  Device-side, no host sync."""
        g = st.flat.grad
        if self._dp_sidx is None or self._dp_sidx.device != g.device:
            self._dp_sidx = torch.arange(0, g.numel(), 64, device=g.device)
        sub = torch.nan_to_num(g.index_select(0, self._dp_sidx), nan=0.0, posinf=0.0, neginf=0.0)
        # unit directions, replicas already excluded (flag / non-finite / norm outlier) left out of
        # the reference: a x50 replica must not define "the others' direction"
        unit = sub / torch.clamp(sub.norm(), min=1e-30)
        contrib = unit * (1.0 - bad_me)
        tot = contrib.clone()
        dist.all_reduce(tot, group=self.dp_group)
        others = tot - contrib
        cos = ((unit * others).sum() / torch.clamp(others.norm(), min=1e-30)).reshape(1)
        allc = [torch.zeros_like(cos) for _ in range(n)]
        dist.all_gather(allc, cos, group=self.dp_group)
        c = torch.cat(allc)
        self._dp_cos = c
        return ((c < 0) & (c < c.median() - float(self.cfg.direction_margin))).float()

    @torch.no_grad()
    def _audit_params(self):
        """Cross-replica weight audit: replicas must hold bit-identical fp32 master weights.  A
        replica whose digest (float64 sum, sum of squares) differs from the majority of its stage
        position was tampered with (parameter perturbation / model poisoning): every rank sees the
        same all-gathered digests, so every rank records it and marks the node compromised in the
        device trust state identically; the stage's replicas then re-synchronise (fp32 master and
        AdamW moments broadcast from a majority member).  One small host read every few steps."""
        st = self.my_stage()
        if st is not None:
            m = st.flat.master.double()
            dg = torch.stack([m.sum(), (m * m).sum()])
        else:
            dg = torch.zeros(2, dtype=torch.float64, device=self.device)
        G = all_gather_rows(dg, self.world)
        note_host_sync()
        G = G.cpu()
        my_pos = self.rank % self.pp
        for pos in range(self.pp):
            ranks = [d * self.pp + pos for d in range(self.dp)]
            rows = [tuple(G[r].tolist()) for r in ranks]
            counts: Dict[tuple, int] = {}
            for r in rows:
                counts[r] = counts.get(r, 0) + 1
            majority, votes = max(counts.items(), key=lambda kv: kv[1])
            divergent = [ranks[i] for i, r in enumerate(rows) if r != majority]
            if not divergent:
                continue
            src = ranks[rows.index(majority)] if votes * 2 > len(ranks) else None
            rec = {"step": self.global_step, "timestamp": time.time(), "attack_type": "model_poisoning",
                   "divergent_nodes": divergent, "resync_from": src, "stage_position": pos}
            self.dp_audits.append(rec)
            logger.warning("parameter audit: replicas %s diverge from the majority (resync from %s)", divergent, src)
            for n in divergent:
                self.attack_history.append({"node_id": n, "timestamp": rec["timestamp"], "step": self.global_step,
                                            "attack_type": "model_poisoning", "ground_truth": None})
                self.trust.mark_compromised(n, "model_poisoning")
                self.t_values[n] = 0.1
                self.t_status[n] = STATUS_CODES[NodeStatus.COMPROMISED]
            if pos == my_pos and src is not None and st is not None:
                for buf in st.flat.optimizer_state_tensors():
                    dist.broadcast(buf, src, group=self.dp_group)
                if st.flat.data is not st.flat.master:
                    st.flat.data.copy_(st.flat.master)
                st.param_checksum = None
