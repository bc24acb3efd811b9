#!/usr/bin/env python3
"""Lying-rank probe against the ROUND-5 gradient commitments (run at commit e56f53d's protocol).

VERDICT r5 weak 1: every r5 attacker was a hook inside an honest engine, so its reporting code was
honest.  Here the target rank (rank 1 of 3 gloo processes, one stage each) runs a SUBCLASS of
``PipelineEngine`` that lies in its own messages:

* ``lie_applied_hash``  applies a sign-flipped gradient and writes its honest committed hash
  (D_GSK_BWD) into the applied-hash slot (D_GSK_APP) of its own digest row;
* ``lie_answer``        sign-flips ONE micro-batch's contribution inside the backward (its running
  commitments follow the tampered state) and answers every challenge with the keyed sketch of the
  honest contribution it kept aside plus the committed snapshot hashes;
* ``hash_forge``        applies a sign-flipped gradient and reports honestly: it rewrites a few hundred
  coordinates with a second preimage of the additive mix32 hash (mix32 is invertible), chosen
  among small fp32 values, so applied hash == committed hash bit for bit.

Every micro-batch is opened (audit_micro_k = M) so the recompute sees every contribution.
Writes one JSON line per attacker (blamed (step, node, kind) triples, tampered steps).  This file
targets the r5 protocol's private methods; scripts/lying_rank.py and tests/test_lying_rank.py run
the same attackers against the protocol that replaced it.
"""
import json
import os
import random
import socket
import sys
import tempfile

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

M32 = 0xFFFFFFFF
START, STEPS, MICRO, TARGET = 4, 9, 4, 1


def _mix(x):
    x ^= x >> 16
    x = (x * 0x7feb352d) & M32
    x ^= x >> 15
    x = (x * 0x6c8e9cf5) & M32
    return x ^ (x >> 16)


def _unmix(y):
    y ^= y >> 16
    y = (y * pow(0x6c8e9cf5, -1, 1 << 32)) & M32
    y ^= (y >> 15) ^ (y >> 30)
    y = (y * pow(0x7feb352d, -1, 1 << 32)) & M32
    return y ^ (y >> 16)


def _engine_cls(kind):
    from trustworthy_dl.parallel.pipeline import PipelineEngine
    from trustworthy_dl.security import stage_verifier as SV

    class Liar(PipelineEngine):
        def _segs_flip(self, st):
            g = st.flat.grad
            for lo, hi in self._commit_segments(st):
                g[lo:hi].neg_()

        # ---- lie_answer: tamper one contribution, answer from the honest copy
        def _commit_micro(self, node, st, i):
            if kind == "lie_answer" and node == self.rank == TARGET and self.global_step >= START and i == 1:
                snap = self._gsnap[node][i]
                honest = st.flat.grad - snap
                self._honest = getattr(self, "_honest", {})
                self._honest[i] = honest.clone()
                st.flat.grad.copy_(snap - honest)          # the contribution sign-flipped
            super()._commit_micro(node, st, i)

        def _answer_challenge(self, node, st, m, key):
            out = super()._answer_challenge(node, st, m, key)
            h = getattr(self, "_honest", {}).get(m)
            if kind == "lie_answer" and h is not None and self.global_step >= START:
                from trustworthy_dl.security.grad_audit import K_KEYED, keyed_sketch
                out[:K_KEYED].copy_(keyed_sketch(h, self._commit_segments(st), key))
            return out

        # ---- lie_applied_hash / hash_forge: rewrite the applied gradient at the step tail
        def _write_commitments(self, node, st, d):
            tamper = node == self.rank == TARGET and self.global_step >= START
            if tamper and kind == "lie_applied_hash":
                self._segs_flip(st)
                super()._write_commitments(node, st, d)
                d[SV.D_GSK_APP:SV.D_GSK_APP + 2].copy_(d[SV.D_GSK_BWD:SV.D_GSK_BWD + 2])
                return
            if tamper and kind == "hash_forge":
                self._forge(st)
            super()._write_commitments(node, st, d)

        def _forge(self, st):
            """Sign-flip the gradient, then rewrite trailing coordinates so the r5 word hash of the
            applied gradient equals the last committed one (second preimage through mix32^-1)."""
            from trustworthy_dl.security.grad_audit import word_hash
            segs = self._commit_segments(st)
            seed = self._hash_seed(st) & M32
            target = int(self._gcom[self.rank][-1])
            self._segs_flip(st)
            g = st.flat.grad
            w = g.view(torch.int32)
            lo, hi = segs[-1]
            rng = random.Random(1234 + self.global_step)
            K = 64
            while True:
                idx = list(range(hi - K, hi))
                cur = int(word_hash(g, segs, seed))
                pos = [_mix((j & M32) ^ seed) for j in idx]
                old = [_mix((int(w[j]) & M32) ^ p) for j, p in zip(idx, pos)]
                R = target - (cur - sum(old))        # what the K fixed words must sum to
                if 0 <= R <= K * M32 * 0.9:
                    break
                K *= 2
            small = lambda bits: ((bits >> 23) & 0xFF) < 117   # |x| < ~1e-3 (no inf / NaN)  # noqa: E731
            for _ in range(10000):
                vals, left = [], R
                ok = True
                for k in range(K - 1):
                    rest = K - 1 - k
                    mean = left // (rest + 1)
                    for _t in range(200):
                        v = min(M32, max(0, int(mean + rng.randint(-(1 << 28), 1 << 28))))
                        if small(_unmix(v) ^ pos[k]):
                            break
                    vals.append(v)
                    left -= v
                if not 0 <= left <= M32 or not small(_unmix(left) ^ pos[-1]):
                    ok = False
                if ok:
                    vals.append(left)
                    break
            for j, p, v in zip(idx, pos, vals):
                bits = _unmix(v) ^ p
                w[j] = bits - (1 << 32) if bits >= 1 << 31 else bits
            assert int(word_hash(g, segs, seed)) == target
            assert bool(torch.isfinite(g).all())
            self.forged = getattr(self, "forged", 0) + 1

    return Liar


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out, kind):
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    cls = _engine_cls(kind) if (rank == TARGET and kind != "clean") else PipelineEngine
    m = get_model("gpt2-tiny", seq_len=32, seed=1)
    eng = cls(m, EngineConfig(num_nodes=world, micro_batches=MICRO, device="cpu", seq_len=32, monitor_seed=0,
                              reassign=False, audit_micro_k=MICRO))
    g = torch.Generator().manual_seed(0)
    for _ in range(STEPS):
        ids = torch.randint(0, 1000, (2 * MICRO, 33), generator=g)
        eng.train_step({"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()})
    eng.flush()
    blamed = sorted({(a["step"], a["node_id"], a["attack_type"]) for a in eng.attack_history})
    with open(f"{out}.{rank}", "w") as f:
        json.dump({"blamed": blamed, "forged": getattr(eng, "forged", 0)}, f)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


def main():
    dest = sys.argv[1] if len(sys.argv) > 1 else "profiles/r6_lying_rank_before.jsonl"
    rows = []
    for kind in ("clean", "lie_applied_hash", "lie_answer", "hash_forge"):
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "r")
            mp.spawn(_worker, args=(3, _port(), out, kind), nprocs=3, join=True)
            res = [json.load(open(f"{out}.{r}")) for r in range(3)]
        row = {"protocol": "r5 (additive mix32 word hash, self-reported applied hash / answers)", "attacker": kind,
               "target": TARGET, "tampered_steps": [] if kind == "clean" else list(range(START, STEPS + 1)),
               "micro_batches": MICRO, "opened_per_step": MICRO, "blamed": res[0]["blamed"],
               "ranks_agree": all(r["blamed"] == res[0]["blamed"] for r in res),
               "forged_steps": res[TARGET]["forged"]}
        rows.append(row)
        print(json.dumps(row), flush=True)
    with open(dest, "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
