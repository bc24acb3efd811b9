"""Trusted shadow snapshots of every stage held by the next stages of the ring:
the source a compromised stage is rebuilt from, so its layers never come from its own memory.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..core.trust_manager import NodeStatus, STATUS_CODES
from ..ops import stats as dstats
from ..runtime.commcheck import note_host_sync
from .comm import all_gather_rows, batched_transfer


class ShadowMixin:
    """Shadow snapshots (mixed into ``PipelineEngine``)."""

    # ================================================================== trusted shadow snapshots
    # SURVEY 5 ("shadow copies of each stage's weights on a neighbour GPU"): when the stages are
    # (re)built and every ``shadow_interval`` steps each stage packs its layers (fp32 master + AdamW
    # moments + buffers, the migration format) and sends them over xGMI to the next
    # ``shadow_copies`` stages of the ring, which keep the copies in HBM (~0.5 GB per GPT-2-medium
    # stage).  The owner's checksum of the packed vector is recorded on every rank.  A periodic
    # copy is committed only when that step's report shows the stage unflagged (the build-time
    # copy at once: the weights come from initialisation, a checkpoint or trusted sources).  A
    # stage later marked compromised is rebuilt from a committed copy held by a trusted holder
    # whose bytes still match the owner's checksum — never from its own (possibly tampered)
    # memory; with no such copy its layers restart from their initial weights.  Metadata (step,
    # layer range, holders, owner checksum) is identical on every rank; only holders keep data.
    def _reset_shadows(self):
        # owner -> committed (step, layer range, primary holder, holders)
        self._shadow_meta: Dict[int, Tuple[int, Tuple[int, int], int, List[int]]] = {}
        self._shadow_pend_meta: Dict[int, Tuple[int, Tuple[int, int], int, List[int]]] = {}
        self._shadow_data: Dict[int, torch.Tensor] = {}      # owner -> committed vector (holders only)
        self._shadow_pend: Dict[int, Tuple[int, torch.Tensor]] = {}
        self._shadow_hash: Dict[int, torch.Tensor] = {}      # owner -> committed owner checksum (every rank)
        self._shadow_pend_hash: Dict[int, torch.Tensor] = {}

    def _shadow_enabled(self) -> bool:
        return self.cfg.shadow_interval > 0 and self.dp == 1 and self.plan.num_stages > 1

    def _shadow_holders(self, node: int) -> List[int]:
        ranks = self.plan.ranks
        i = ranks.index(node)
        k = max(1, min(int(self.cfg.shadow_copies), len(ranks) - 1))
        return [ranks[(i + d) % len(ranks)] for d in range(1, k + 1)]

    def _shadow_holder(self, node: int) -> int:
        return self._shadow_holders(node)[0]

    def _shadow_usable(self, c: int, bad: Sequence[int] = ()) -> bool:
        return self._shadow_source(c, bad) is not None

    def _shadow_source(self, c: int, bad: Sequence[int] = (), verified: Optional[Dict] = None) -> Optional[int]:
        """The holder that serves owner ``c``'s committed copy: the first of its holders that is
        not excluded, not among ``bad`` (the nodes being compromised now), may take tasks and (when
        ``verified`` is given) whose copy still matches the owner's checksum."""
        meta = self._shadow_meta.get(c)
        if meta is None:
            return None
        for h in meta[3]:
            if h in self.excluded or h in bad or not self.trust.can_assign_task(h):
                continue
            if verified is not None and not verified.get((c, h), False):
                continue
            return h
        return None

    def _verify_shadows(self) -> Dict[Tuple[int, int], bool]:
        """(owner, holder) -> the holder's committed copy matches the owner's checksum.  Each rank
        checks the copies it holds; distributed: one all-gather so every rank decides alike."""
        N = self.num_nodes
        mine = torch.zeros(N, dtype=torch.float32, device=self.device)
        for c, vec in self._shadow_data.items():
            ref = self._shadow_hash.get(c)
            if ref is not None:
                ok = torch.equal(dstats.checksum(vec).to(ref.device), ref)
                mine[c] = 1.0 if ok else 0.0
        out: Dict[Tuple[int, int], bool] = {}
        if self.distributed:
            V = all_gather_rows(mine, self.world)
            note_host_sync()
            V = V.cpu()
            for c, meta in self._shadow_meta.items():
                for h in meta[3]:
                    out[(c, h)] = bool(V[h, c] > 0)
        else:
            for c, meta in self._shadow_meta.items():
                for h in meta[3]:
                    out[(c, h)] = bool(mine[c] > 0)
        return out

    def _shadow_slice(self, li: int) -> torch.Tensor:
        for c, meta in self._shadow_meta.items():
            a, b = meta[1]
            if a <= li < b:
                off = sum(self._packed_numel(k) for k in range(a, li))
                return self._shadow_data[c][off:off + self._packed_numel(li)]
        raise KeyError(li)

    @torch.no_grad()
    def _take_shadow(self):
        step = self.global_step
        owners = list(self.plan.ranks)
        for node, rng in zip(self.plan.ranks, self.plan.ranges):
            hs = self._shadow_holders(node)
            self._shadow_pend_meta[node] = (step, tuple(rng), hs[0], hs)
        if self.distributed:
            st = self.my_stage()
            vec = (torch.cat([self._pack_layer(st, li) for li in range(*st.layer_range)]) if st is not None
                   else torch.zeros(0, device=self.device))
            h = dstats.checksum(vec) if st is not None else torch.zeros(3, dtype=torch.float64, device=self.device)
            H = all_gather_rows(h, self.world)
            for node in owners:
                self._shadow_pend_hash[node] = H[node].clone()
            if st is None:
                return
            sends = [(vec, hd) for hd in self._shadow_holders(self.rank)]
            recvs = []
            for o in owners:
                if o != self.rank and self.rank in self._shadow_holders(o):
                    a, b = self.plan.ranges[owners.index(o)]
                    buf = torch.empty(sum(self._packed_numel(li) for li in range(a, b)), dtype=torch.float32,
                                      device=self.device)
                    recvs.append((buf, o))
                    self._shadow_pend[o] = (step, buf)
            self._note_peers(sends, recvs)
            batched_transfer(sends, recvs, meter=self.link_meter)
        else:
            for node, st in self.stages.items():
                dev = self.stages[self._shadow_holder(node)].device
                vec = torch.cat([self._pack_layer(st, li) for li in range(*st.layer_range)])
                self._shadow_pend_hash[node] = dstats.checksum(vec)
                self._shadow_pend[node] = (step, vec.to(dev, copy=True))

    def refresh_shadows(self):
        """Take and commit a snapshot now (stages freshly built from trusted weights: at start-up,
        after a re-shard, after a checkpoint load), so a committed copy exists from step 0 on."""
        if not self._shadow_enabled():
            return
        self._reset_shadows()
        self._take_shadow()
        for owner in list(self._shadow_pend_meta):
            self._commit_one(owner, self.global_step)

    def _commit_one(self, owner: int, step: int) -> None:
        meta = self._shadow_pend_meta.pop(owner)
        data = self._shadow_pend.pop(owner, None)
        if data is not None and data[0] != step:   # a newer snapshot replaced it: keep that one
            self._shadow_pend[owner] = data
            data = None
        self._shadow_meta[owner] = meta
        if owner in self._shadow_pend_hash:
            self._shadow_hash[owner] = self._shadow_pend_hash.pop(owner)
        if data is not None:
            self._shadow_data[owner] = data[1]

    def _commit_shadows(self, step: int, blamed: Sequence[bool], statuses: Sequence[int]):
        bad = (STATUS_CODES[NodeStatus.COMPROMISED], STATUS_CODES[NodeStatus.SUSPICIOUS])
        for owner, meta in list(self._shadow_pend_meta.items()):
            if meta[0] != step:
                continue
            if blamed[owner] or statuses[owner] in bad:
                self._shadow_pend_meta.pop(owner)
                data = self._shadow_pend.pop(owner, None)
                if data is not None and data[0] != step:
                    self._shadow_pend[owner] = data
                self._shadow_pend_hash.pop(owner, None)
                continue
            self._commit_one(owner, step)
