#!/usr/bin/env python3
"""Attack configurations through the DISTRIBUTED engine: one process per pipeline stage (gloo on
CPU here; the same code path runs RCCL on GPUs), detection only, so every injection is scored.

The GPU attack-config records (scripts/run_attack_configs.py) run the engine in local mode on one
MI355X; this runs the multi-rank protocol itself — the commit-before-reveal gradient sketches, the
private audit choice revealed through the c10d store, the weight / input / gradient shipment to the
auditor, the cross-checked hashes and the all-gathered digest — and scores it the same way
(reference scoring: /root/reference/experiment_runner.py:84-112; attacks:
/root/reference/adversarial_attacks.py).  Every rank computes the same blame from the same
all-gathered digests; rank 0 writes one JSON line per run.

  python scripts/run_attack_configs_dist.py --configs signflip,dx,last,liar,byz1m,clean --seeds 1,2 \\
      --out profiles/r4_cfg_dist_gloo.jsonl
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

CONFIGS = {
    "signflip": dict(attack=dict(attack_types=["gradient_poisoning"], gradient_mode="sign_flip"), targets=[3]),
    "dx": dict(attack=dict(attack_types=["byzantine_backward"], intensity=0.5), targets=[4]),
    "last": dict(attack=dict(attack_types=["byzantine_backward"], intensity=0.5), targets=[7]),
    "liar": dict(attack=dict(attack_types=["model_poisoning"], intensity=0.05, lie_integrity=True), targets=[6]),
    "byz1m": dict(attack=dict(attack_types=["byzantine"], intensity=0.5, micro_batches=1), targets=[2],
                  cfg=dict(audit_targeted=True)),
    # round 5: adaptive attacker (knows the job seed; hides from the public sketch window): rewrite after
    # the backward / one micro-batch's contribution inside it, k = 2 of M = 8 audited per step
    "adapt": dict(attack=dict(attack_types=["gradient_poisoning"], gradient_mode="sign_flip", adaptive=True),
                  targets=[3]),
    "adapt1m": dict(attack=dict(attack_types=["gradient_poisoning"], gradient_mode="sign_flip", adaptive=True,
                                micro_batches=1), targets=[3], cfg=dict(audit_micro_k=2)),
    "clean": dict(attack=None, targets=[]),
}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out, cfg_id, seed, a):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from trustworthy_dl.attacks.adversarial_attacks import AdversarialAttacker, AttackConfig
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    c = CONFIGS[cfg_id]
    att = None
    if c["attack"]:
        att = AdversarialAttacker(AttackConfig(target_nodes=list(c["targets"]), start_step=a.start,
                                               probability=a.p_attack, seed=seed, **c["attack"]))
        att.activate_attacks()
    model = get_model(a.model, seq_len=a.seq_len, seed=1, vocab_size=a.vocab)
    ecfg = EngineConfig(num_nodes=world, micro_batches=a.batch // a.mbs, device="cpu", seq_len=a.seq_len,
                        monitor_seed=seed, reassign=False, **c.get("cfg", {}))
    eng = PipelineEngine(model, ecfg, attacker=att)
    g = torch.Generator().manual_seed(seed)
    t0 = time.time()
    for step in range(a.steps):
        ids = torch.randint(0, a.vocab, (a.batch, a.seq_len + 1), generator=g)
        eng.train_step({"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()})
        if rank == 0 and (step + 1) % 20 == 0:
            print(f"[{cfg_id} seed {seed}] step {step + 1}/{a.steps} {time.time() - t0:.0f}s", flush=True)
    eng.flush()
    wall = time.time() - t0
    inj = att.injections if att is not None else []
    mine = {"tampered": sorted({(i["node"], i["step"]) for i in inj}), "n_inj": len(inj)}
    allm = [None] * world
    dist.all_gather_object(allm, mine)
    if rank == 0:
        tampered = sorted({tuple(t) for m in allm for t in m["tampered"]})
        blamed = sorted({(r["step"], r["node_id"], r["attack_type"]) for r in eng.attack_history})
        det = att.detection_metrics() if att is not None else {}
        rec = {"config": cfg_id, "seed": seed, "mode": "distributed (gloo, one process per stage)", "world": world,
               "model": a.model, "seq_len": a.seq_len, "batch": a.batch, "micro_batches": a.batch // a.mbs,
               "steps": a.steps, "attack_start": a.start, "p_attack": a.p_attack, "targets": c["targets"],
               "attack": c["attack"], "injections": sum(m["n_inj"] for m in allm),
               "tampered_steps": len(tampered),
               "detection": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in det.items()
                             if k in ("tp", "fp", "fn", "precision", "recall", "f1")},
               "blamed_nodes": sorted({n for _, n, _ in blamed}),
               "clean_nodes_blamed": sorted({n for _, n, _ in blamed if n not in c["targets"]}),
               "tampered_steps_caught": len({(n, s) for s, n, _ in blamed} & set(tampered)),
               "evidence_kinds": sorted({k for _, _, k in blamed}),
               "audit": eng.audit_summary(), "last_loss": eng.last_loss, "wall_s": round(wall, 1)}
        with open(out, "w") as f:
            json.dump(rec, f)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="signflip,dx,last,liar,byz1m,clean")
    ap.add_argument("--seeds", default="1,2")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--model", default="gpt2-mini")
    ap.add_argument("--vocab", type=int, default=1024)
    ap.add_argument("--seq-len", type=int, default=32)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--mbs", type=int, default=2)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--start", type=int, default=10)
    ap.add_argument("--p-attack", type=float, default=0.5)
    ap.add_argument("--out", default="gpurun_out/r4_cfg_dist_gloo.jsonl")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    for cfg_id in a.configs.split(","):
        for seed in [int(s) for s in a.seeds.split(",")]:
            with tempfile.TemporaryDirectory() as td:
                path = os.path.join(td, "rec.json")
                mp.spawn(_worker, args=(a.world, _free_port(), path, cfg_id, seed, a), nprocs=a.world, join=True)
                rec = json.load(open(path))
            with open(a.out, "a") as f:
                f.write(json.dumps(rec) + "\n")
            print(json.dumps({k: rec[k] for k in ("config", "seed", "injections", "tampered_steps", "detection",
                                                   "clean_nodes_blamed", "tampered_steps_caught")}), flush=True)


if __name__ == "__main__":
    main()
