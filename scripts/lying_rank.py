#!/usr/bin/env python3
"""Lying ranks against the round-6 audit protocol on 8 gloo processes (one pipeline stage each).

For each attacker of attacks/lying_rank.py (plus a clean control) and each seed: GPT-2-mini (1k
vocabulary, T = 32), 8 stages, M micro-batches of which the auditors open k per step; the liar is
the PipelineEngine subclass of ONE rank, lying from step 3 on; no re-shard (the liar keeps lying, so
every lying step is scored).  One JSON line per run: the lying steps (the liar's ground truth), the
blamed (step, node, kind) triples every rank agreed on, per-step catch rate vs k / M, clean blames.

    python scripts/lying_rank.py --out profiles/r6_lying_rank_gloo8.jsonl --seeds 1,2,3
"""
import argparse
import json
import os
import socket
import sys
import tempfile
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out, kind, target, micro, k, steps, seed, start):
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from trustworthy_dl.attacks.lying_rank import make_lying_engine
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    cls = make_lying_engine(PipelineEngine, kind, target=target, start=start, seed=seed) \
        if kind != "clean" and rank == target else PipelineEngine
    m = get_model("gpt2-mini", seq_len=32, seed=1, vocab_size=1024)
    eng = cls(m, EngineConfig(num_nodes=world, micro_batches=micro, device="cpu", seq_len=32, monitor_seed=seed,
                              reassign=False, audit_micro_k=k, audit_targeted=False))
    g = torch.Generator().manual_seed(seed)
    t0 = time.perf_counter()
    for _ in range(steps):
        ids = torch.randint(0, 1000, (2 * micro, 33), generator=g)
        eng.train_step({"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()})
    eng.flush()
    dt = time.perf_counter() - t0
    blamed = sorted({(a["step"], a["node_id"], a["attack_type"]) for a in eng.attack_history})
    with open(f"{out}.{rank}", "w") as f:
        json.dump({"blamed": blamed, "lied": getattr(eng, "lied_steps", []), "audit": eng.audit_summary(),
                   "s_per_step": dt / steps, "loss": eng.last_loss}, f)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--micro", type=int, default=8)
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--start", type=int, default=3)
    ap.add_argument("--target", type=int, default=3)
    ap.add_argument("--seeds", default="1,2,3")
    ap.add_argument("--attacks", default="clean,lie_applied,lie_answer,hash_forge")
    ap.add_argument("--out", default="profiles/r6_lying_rank_gloo8.jsonl")
    a = ap.parse_args()
    for seed in [int(s) for s in a.seeds.split(",")]:
        for kind in a.attacks.split(","):
            with tempfile.TemporaryDirectory() as td:
                out = os.path.join(td, "r")
                mp.spawn(_worker, args=(a.world, _port(), out, kind, a.target, a.micro, a.k, a.steps, seed, a.start),
                         nprocs=a.world, join=True)
                res = [json.load(open(f"{out}.{r}")) for r in range(a.world)]
            blamed = res[0]["blamed"]
            lied = res[a.target]["lied"] if kind != "clean" else []
            caught = sorted({s for s, n, _ in blamed if n == a.target})
            row = {"protocol": "r6 (BLAKE2s Merkle commitments, key after commit, open after sketches, live "
                               "optimizer mirror)",
                   "attacker": kind, "seed": seed, "world": a.world, "target": a.target, "micro_batches": a.micro,
                   "opened_per_step": a.k, "k_over_m": a.k / a.micro, "lied_steps": lied,
                   "blamed": blamed, "ranks_agree": all(r["blamed"] == blamed for r in res),
                   "clean_blames": [b for b in blamed if b[1] != a.target],
                   "caught_steps": caught,
                   "catch_rate_per_lying_step": (len(set(caught) & set(lied)) / len(lied)) if lied else None,
                   "first_caught": caught[0] if caught else None,
                   "auditor_of_target": res[a.target + 1]["audit"] if a.target + 1 < a.world else None,
                   "s_per_step": max(r["s_per_step"] for r in res)}
            print(json.dumps({k: v for k, v in row.items() if k not in ("blamed", "auditor_of_target")}), flush=True)
            with open(a.out, "a") as f:
                f.write(json.dumps(row) + "\n")


if __name__ == "__main__":
    main()
