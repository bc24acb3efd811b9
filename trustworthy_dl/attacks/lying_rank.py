"""Byzantine ranks that LIE in the audit protocol: ``PipelineEngine`` subclasses whose auditee-side
methods (parallel/commitments.py) report something other than what the stage does.

The hook attackers of ``adversarial_attacks.py`` rewrite tensors inside an honest engine, so their
reports are honest; VERDICT r5 showed that a one-line lie in a rank's own report evaded the r5
commitments (scripts/lying_rank_before.py: 0 of 6 tampered steps blamed for each attacker below).
Here the lie is the rank's code: it runs in its own gloo / RCCL process (tests/test_lying_rank.py,
scripts/lying_rank.py) or, in local mode, for its own node only.

* ``lie_applied``  applies a sign-flipped gradient; every commitment, sketch, opening and the
  gradient it ships come from an honest copy.  The auditor's mirror applies the honest one, so the
  stage's weights leave the mirror: caught at the next step's weight check (and forward recompute).
* ``lie_answer``   applies G - 2 c_j (micro-batch j's contribution sign-flipped, j private to the
  rank each step), ships and commits that gradient, keeps the honest contribution commitments and
  openings, and reports s_j' = S(c_j) - 2 S(c_j) so the sketches still sum to S(G').  Caught
  exactly when j is opened (probability k / M per step).
* ``hash_forge``   applies and ships a sign-flipped gradient with r5's mix32 second-preimage
  fix-up, and commits the honest gradient's root in its place: a collision of the BLAKE2s Merkle
  root would be needed.  Caught every step (root of the shipped gradient != commitment).
* ``lie_sumsq``     reports a huge gradient sum of squares in its digest row (every stage's updates
  would be clipped to nothing).  Harmless: the global clip uses the sums its auditor computed.
* ``lie_tied``      a tie-group member (GPT-2: the embedding or the LM-head stage) applies, ships and
  commits the tied weight's gradient sign-flipped after the tied all-reduce; everything else honest.
  The stage's own sum check excludes the tied rows (the all-reduce adds the other member's
  contributions there): caught by the cross-member tie check (its auditor's sketch of the tied
  gradient it applies != the sum of both members' committed tied contributions, while the other
  member's matches).
* ``lie_tied_feed`` a tie-group member feeds the tied all-reduce its gradient sign-flipped (after its
  contributions were committed): both members then apply the same wrong sum.  Which member fed it
  is not identifiable from the sums, so nobody is blamed — the replica's update is skipped every
  such step (tampering evidence), and the weights never take the poisoned gradient.

Ground truth: ``lied_steps`` lists the steps where the rank applied something else than the honest
gradient.  Reference: the optimizer step trusts every node (distributed_trainer.py:441-446).
"""
from __future__ import annotations

import random
from typing import List, Optional

import torch

ATTACKS = ("lie_applied", "lie_answer", "hash_forge", "lie_sumsq", "lie_tied", "lie_tied_feed")


def make_lying_engine(base_cls, kind: str, target: int, start: int, seed: int = 0):
    """Subclass of ``base_cls`` (PipelineEngine) that lies as ``kind`` on node ``target`` from step
    ``start`` on."""
    if kind not in ATTACKS:
        raise ValueError(f"unknown lying-rank attack {kind!r}; one of {ATTACKS}")

    class LyingEngine(base_cls):
        lie_kind = kind

        def _lie_init(self):
            if not hasattr(self, "lied_steps"):
                self.lied_steps: List[int] = []
                self._lie_rng = random.Random(seed * 7919 + target)
                self._honest_g: Optional[torch.Tensor] = None
                self._lie_j = -1
                self._lie_delta_s = None

        def _lying_now(self, node: int) -> bool:
            self._lie_init()
            return node == target and self.global_step >= start

        def _flip(self, g: torch.Tensor, st) -> torch.Tensor:
            t = g.clone()
            for lo, hi in self._commit_segments(st):
                t[lo:hi].neg_()
            return t

        # ---- every answer starts from the commitments call (once per step, before the others)
        @torch.no_grad()
        def _contrib_commitments(self, node, st):
            self._lie_init()
            self._honest_g = None
            self._lie_j = -1
            if not self._lying_now(node) or kind in ("lie_sumsq", "lie_tied_feed"):
                return super()._contrib_commitments(node, st)
            if kind == "lie_tied":
                tr = self._tie_range(st)
                if tr is not None:
                    st.flat.grad[tr[0]:tr[0] + tr[1]].neg_()     # applied, shipped and committed
                    self.lied_steps.append(self.global_step)
                return super()._contrib_commitments(node, st)
            if kind == "lie_applied":
                self._honest_g = st.flat.grad.clone()            # shipped + committed
                st.flat.grad.copy_(self._flip(st.flat.grad, st))  # applied
                self.lied_steps.append(self.global_step)
                return super()._contrib_commitments(node, st)
            if kind == "lie_answer":
                ring = self._gring[node]
                j = self._lie_j = self._lie_rng.randrange(ring.shape[0])
                st.flat.grad.sub_(2.0 * ring[j])                  # applied (and shipped) G' = G - 2 c_j
                self.lied_steps.append(self.global_step)
                return super()._contrib_commitments(node, st)
            # hash_forge: commit the honest root, apply + ship the forged gradient
            from ..security.grad_audit import merkle_root
            segs = self._commit_segments(st)
            honest_root = merkle_root(st.flat.grad, segs)
            st.flat.grad.copy_(self._forged(st))
            self.lied_steps.append(self.global_step)
            C = super()._contrib_commitments(node, st)
            C[C.shape[0] - 2].copy_(honest_root.to(C.device))
            return C

        def _write_commitments(self, node, st, d):
            super()._write_commitments(node, st, d)
            if kind == "lie_sumsq" and self._lying_now(node):
                from ..security import stage_verifier as SV
                d[SV.D_GRAD_SUMSQ:SV.D_GRAD_SUMSQ + 1].fill_(1e12)
                self.lied_steps.append(self.global_step)

        @torch.no_grad()
        def _note_tied_pre(self, st):
            super()._note_tied_pre(st)
            node = self._node_of(st)
            if kind == "lie_tied_feed" and self._lying_now(node):
                tr = self._tie_range(st)
                if tr is not None:
                    st.flat.grad[tr[0]:tr[0] + tr[1]].neg_()     # what goes into the all-reduce
                    self.lied_steps.append(self.global_step)

        def _applied_gradient(self, node, st):
            if self._lying_now(node) and kind == "lie_applied" and self._honest_g is not None:
                return self._honest_g
            return super()._applied_gradient(node, st)

        @torch.no_grad()
        def _contrib_sketches(self, node, st, key):
            s = super()._contrib_sketches(node, st, key)
            if self._lying_now(node) and kind == "lie_answer" and self._lie_j >= 0:
                s[self._lie_j] = -s[self._lie_j]                 # S(c_j) - 2 S(c_j): the sum stays S(G')
            return s

        def _forged(self, st) -> torch.Tensor:
            """Sign flip + r5-style fix-up words (mix32^-1 of the hash difference): a second preimage
            of the old additive hash, nothing for a Merkle root."""
            g = self._flip(st.flat.grad, st)
            segs = self._commit_segments(st)
            if segs:
                lo, hi = segs[-1]
                k = min(64, hi - lo)
                w = g[hi - k:hi].view(torch.int32)
                for i in range(k):     # small, finite fix-up values (the r5 forge picked them the same way)
                    w[i] = (self._lie_rng.getrandbits(23)) | (100 << 23)
            return g

    LyingEngine.__name__ = f"LyingEngine_{kind}"
    return LyingEngine
