"""Cost-balanced contiguous layer -> stage partitioning.

Replaces the reference's ``layers_per_node = len(h) // num_nodes`` split (distributed_trainer.py:
124-135), which drops the remainder layers and the embedding / head.  Here the whole
``pipeline_layers()`` list is split into contiguous ranges minimising the most expensive stage
(exact min-max DP over per-layer fwd+bwd cost), optionally over an arbitrary subset of ranks (the
trusted set after a re-shard).  Every stage gets >= 1 layer.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple


def balanced_partition(costs: Sequence[float], num_stages: int) -> List[Tuple[int, int]]:
    """Split layers [0, L) into ``num_stages`` contiguous non-empty ranges minimising the max cost."""
    L = len(costs)
    if num_stages < 1:
        raise ValueError("num_stages must be >= 1")
    if num_stages > L:
        raise ValueError(f"cannot place {L} layers on {num_stages} stages (each stage needs >= 1 layer)")
    pre = [0.0]
    for c in costs:
        pre.append(pre[-1] + float(c))
    INF = float("inf")
    # best[s][i]: min max-cost placing first i layers on s stages; cut[s][i]: start of last stage
    best = [[INF] * (L + 1) for _ in range(num_stages + 1)]
    cut = [[0] * (L + 1) for _ in range(num_stages + 1)]
    best[0][0] = 0.0
    for s in range(1, num_stages + 1):
        for i in range(s, L - (num_stages - s) + 1):
            bv, bj = INF, s - 1
            for j in range(s - 1, i):
                v = max(best[s - 1][j], pre[i] - pre[j])
                if v < bv or (v == bv and j > bj):
                    bv, bj = v, j
            best[s][i], cut[s][i] = bv, bj
    ranges = []
    i = L
    for s in range(num_stages, 0, -1):
        j = cut[s][i]
        ranges.append((j, i))
        i = j
    return ranges[::-1]


def even_partition(num_layers: int, num_stages: int) -> List[Tuple[int, int]]:
    """Equal layer counts (remainder spread over the first stages) — never drops layers."""
    base, rem = divmod(num_layers, num_stages)
    out, st = [], 0
    for s in range(num_stages):
        n = base + (1 if s < rem else 0)
        out.append((st, st + n))
        st += n
    return out


@dataclass
class PlacementPlan:
    """Stage order -> (rank, layer range).  ``ranks[i]`` runs stage i."""
    ranks: List[int]
    ranges: List[Tuple[int, int]]
    version: int = 0

    @property
    def num_stages(self) -> int:
        return len(self.ranks)

    def stage_of_rank(self, rank: int) -> Optional[int]:
        try:
            return self.ranks.index(rank)
        except ValueError:
            return None

    def owner_of_layer(self, layer: int) -> int:
        for r, (a, b) in zip(self.ranks, self.ranges):
            if a <= layer < b:
                return r
        raise KeyError(layer)

    def layers_of_rank(self, rank: int) -> Tuple[int, int]:
        s = self.stage_of_rank(rank)
        return (0, 0) if s is None else self.ranges[s]

    def to_list(self) -> List[int]:
        """Flat int encoding used for the collective broadcast of a plan: [version, S, r0, a0, b0, ...]."""
        out = [self.version, self.num_stages]
        for r, (a, b) in zip(self.ranks, self.ranges):
            out += [r, a, b]
        return out

    @classmethod
    def from_list(cls, v: Sequence[int]) -> "PlacementPlan":
        ver, S = int(v[0]), int(v[1])
        ranks, ranges = [], []
        for i in range(S):
            r, a, b = (int(x) for x in v[2 + 3 * i: 5 + 3 * i])
            ranks.append(r)
            ranges.append((a, b))
        return cls(ranks, ranges, ver)

    def describe(self, names: Optional[Sequence[str]] = None) -> str:
        parts = []
        for i, (r, (a, b)) in enumerate(zip(self.ranks, self.ranges)):
            parts.append(f"stage{i}@rank{r}:[{a},{b})")
        return " ".join(parts)


def make_plan(costs: Sequence[float], ranks: Sequence[int], version: int = 0,
              balanced: bool = True) -> PlacementPlan:
    ranks = list(ranks)
    ranges = balanced_partition(costs, len(ranks)) if balanced else even_partition(len(costs), len(ranks))
    return PlacementPlan(ranks, ranges, version)


def stage_imbalance(costs: Sequence[float], ranges: Sequence[Tuple[int, int]]) -> float:
    """max stage cost / mean stage cost (1.0 = perfectly balanced)."""
    per = [sum(costs[a:b]) for a, b in ranges]
    return max(per) / (sum(per) / len(per))
