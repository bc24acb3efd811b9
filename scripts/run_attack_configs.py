#!/usr/bin/env python3
"""BASELINE.json attack configurations 3 / 4 / 5, end to end in local mode (every stage on one GPU).

    3  GPT-2-medium, 8 stages, gradient poisoning on one stage -> detection -> re-shard to 7
    4  ResNet-50,    8 stages, parameter perturbation on one stage -> detection -> reassignment
    5  GPT-2-medium, 8 stages, 2 Byzantine (activation-tampering) stages -> re-shard to 6

Training data is the learnable synthetic stream (Markov tokens / class-conditional images), so
the loss falls while the attack runs.  Per config one JSON record: detection precision / recall /
F1 and time-to-detect (attacker ground truth vs the engine's per-stage verdicts), the re-shard
wall time (ms, migration of fp32 master + AdamW moments), the plan before / after, final trust,
and the loss curve across the re-shard.  The reference describes these configs
(experiment_runner.py:84-112, README.md:85-92) but never runs a re-shard.

    python scripts/run_attack_configs.py --configs 3,4,5 --out profiles/r2_attack_configs.jsonl
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from trustworthy_dl.attacks.adversarial_attacks import AdversarialAttacker, AttackConfig  # noqa: E402
from trustworthy_dl.models import get_model  # noqa: E402
from trustworthy_dl.parallel.flat import AdamWConfig  # noqa: E402
from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine  # noqa: E402
from trustworthy_dl.utils.data_loader import MarkovLanguageModeling, SyntheticImages  # noqa: E402
from trustworthy_dl.utils.metrics import MetricsCollector  # noqa: E402

CONFIGS = {
    3: dict(model="gpt2-medium", attack=dict(attack_types=["gradient_poisoning"], gradient_mode="scale",
                                             gradient_scale=10.0), targets=[3], lr=1e-4),
    # ImageNet-shape ResNet-50 at the bench's batch (64, micro-batch 8): BatchNorm over 2 images
    # (the r2 first run: batch 8 / micro-batch 2) makes every stage's gradient norm heavy-tailed
    4: dict(model="resnet50", attack=dict(attack_types=["model_poisoning"], intensity=0.05), targets=[4], lr=3e-4,
            batch=64, mbs=8),
    5: dict(model="gpt2-medium", attack=dict(attack_types=["byzantine"], intensity=0.5), targets=[2, 5], lr=1e-4),
}


CONFIGS["clean"] = dict(model="gpt2-medium", attack=None, targets=[], lr=1e-4)
# round 4 (backward audit): sign-flip gradient poisoning (reference F1 0.0), activation-gradient
# (dX) tampering, the loss stage tampering its dX, single-micro-batch (one-of-M) adversaries, and a
# model-poisoning rank that lies about its own integrity check
CONFIGS["3s"] = dict(model="gpt2-medium", attack=dict(attack_types=["gradient_poisoning"], gradient_mode="sign_flip"),
                     targets=[3], lr=1e-4)
CONFIGS["dx"] = dict(model="gpt2-medium", attack=dict(attack_types=["byzantine_backward"], intensity=0.5),
                     targets=[4], lr=1e-4)
CONFIGS["last"] = dict(model="gpt2-medium", attack=dict(attack_types=["byzantine_backward"], intensity=0.5),
                       targets=[7], lr=1e-4)
CONFIGS["3m"] = dict(model="gpt2-medium", attack=dict(attack_types=["gradient_poisoning"], gradient_mode="sign_flip",
                                                      micro_batches=1), targets=[3], lr=1e-4)
CONFIGS["5m"] = dict(model="gpt2-medium", attack=dict(attack_types=["byzantine"], intensity=0.5, micro_batches=1),
                     targets=[2, 5], lr=1e-4)
# one micro-batch's weight-gradient contribution scaled (its committed sketch norm stands out: the
# targeted audit picks it)
CONFIGS["3ms"] = dict(model="gpt2-medium", attack=dict(attack_types=["gradient_poisoning"], gradient_mode="scale",
                                                       micro_batches=1), targets=[3], lr=1e-4)
# round 5 (commit-then-reveal audit): ADAPTIVE gradient poisoning that knows the public job seed and
# hides its sign flip from the public sketch window; "3a" rewrites the gradient after the backward,
# "3am" tampers one micro-batch's contribution inside it (caught by the keyed recompute of an audited
# micro-batch: k of M per step, here k = 4 of 16)
CONFIGS["3a"] = dict(model="gpt2-medium", attack=dict(attack_types=["gradient_poisoning"], gradient_mode="sign_flip",
                                                      adaptive=True), targets=[3], lr=1e-4)
CONFIGS["3am"] = dict(model="gpt2-medium", attack=dict(attack_types=["gradient_poisoning"], gradient_mode="sign_flip",
                                                       adaptive=True, micro_batches=1), targets=[3], lr=1e-4,
                      audit_micro_k=4)
CONFIGS["liar"] = dict(model="gpt2-medium", attack=dict(attack_types=["model_poisoning"], intensity=0.05,
                                                        lie_integrity=True), targets=[6], lr=1e-4)


def run(cfg_id, device: str, steps: int, start: int, batch: int, mbs: int, seq_len: int, p_attack: float,
        small: bool = False, warmup: int = 50, seed: int = 3, reassign: bool = True, audit: bool = True):
    c = dict(CONFIGS[cfg_id])
    batch, mbs = c.get("batch", batch), c.get("mbs", mbs)
    if small:   # CPU smoke: same flow on the tiny models
        c["model"] = {"gpt2-medium": "gpt2-tiny", "resnet50": "resnet32"}[c["model"]]
    att = None
    if c["attack"] is not None:
        att = AdversarialAttacker(AttackConfig(target_nodes=c["targets"], start_step=start, probability=p_attack,
                                               seed=seed, **c["attack"]))
        att.activate_attacks()
    gpt = c["model"].startswith("gpt2")
    img = 32 if c["model"] == "resnet32" else 224
    ncls = 10 if img == 32 else 1000
    model = get_model(c["model"], seq_len=seq_len, seed=5) if gpt else \
        (get_model(c["model"], seed=5) if img == 32 else get_model(c["model"], image_size=img, seed=5))
    extra = {"seq_len": seq_len} if gpt else {}
    cfg = EngineConfig(num_nodes=8, micro_batches=max(1, batch // mbs), device=device,
                       adamw=AdamWConfig(lr=c["lr"], weight_decay=0.01, max_grad_norm=1.0, warmup_steps=20),
                       attack_detection=True, gradient_verification=True, quarantine=True, reassign=reassign,
                       audit=audit,
                       # detector warm-up of 50 clean steps before the attacks start at step 100 (the
                       # reference protocol warms up on 100 clean steps: BASELINE.md); at 20 the
                       # baselines of GPT-2 hidden states caught early-training transients as z ~ 30
                       # output anomalies; the monitored micro-batch RNG is pinned for reproducibility
                       verifier={"warmup": warmup}, monitor_seed=seed, audit_micro_k=c.get("audit_micro_k", 1), **extra)
    eng = PipelineEngine(model, cfg, attacker=att, metrics=MetricsCollector())
    del model
    plan0 = eng.plan.describe()
    data = (MarkovLanguageModeling(batch, seq_len, 8192, num_batches=steps, seed=1) if gpt else
            SyntheticImages(batch, img, ncls, num_batches=steps, seed=1))
    t0 = time.perf_counter()
    for i, b in enumerate(data):
        eng.train_step(b)
        if i % 50 == 49:   # progress (a long run must not look hung)
            print(f"[cfg {cfg_id} seed {seed}] step {i + 1}/{steps} {time.perf_counter() - t0:.0f}s",
                  file=sys.stderr, flush=True)
    eng.flush()
    if device.startswith("cuda"):
        torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    m = att.detection_metrics() if att is not None else {}
    losses = [(r["step"], round(r["loss"], 4)) for r in eng.metrics.batch_metrics if r.get("loss") is not None]
    rs = eng.reassignment_history
    first_attack = min(att.first_attack_step.values()) if att is not None and att.first_attack_step else None
    clean_blamed = sorted({r["node_id"] for r in eng.attack_history if not r.get("ground_truth")})
    # per target: first tampered step, first detection, first re-shard away from it (reports late)
    lag = {}
    for n in c["targets"]:
        inj = sorted(i["step"] for i in (att.injections if att is not None else []) if i["node"] == n)
        det = sorted(r["step"] for r in eng.attack_history if r["node_id"] == n and r.get("ground_truth"))
        rsh = sorted(r["step"] for r in rs if n in r["from_nodes"])
        lag[str(n)] = {"first_tamper": inj[0] if inj else None, "first_detect": det[0] if det else None,
                       "reshard": rsh[0] if rsh else None,
                       "tampered_steps_before_reshard": (len({s for s in inj if s <= rsh[0]}) if inj and rsh else None)}
    compromised = [n for n in range(8) if eng.trust.get_node_status(n).value == "compromised"]
    rec = {
        "config": cfg_id, "seed": seed, "reassign": reassign, "audit": audit,
        "model": c["model"], "attack": c["attack"], "targets": c["targets"],
        "p_attack": p_attack, "attack_start_step": start, "first_attack_step": first_attack, "steps": steps,
        "batch": batch, "micro_batch": mbs, "seq_len": seq_len if gpt else None, "device": device,
        "data": "markov tokens (order 1, branching 4, 8192 ids)" if gpt else "class-conditional synthetic images",
        "lr": c["lr"], "lr_warmup_steps": 20, "detector_warmup": warmup,
        "detection": {k: (round(v, 4) if isinstance(v, float) else v) for k, v in m.items()
                      if k in ("tp", "fp", "fn", "precision", "recall", "f1", "mean_time_to_detect_steps")},
        "injections": len(att.injections) if att is not None else 0,
        "tampered_steps": len({(i["node"], i["step"]) for i in att.injections}) if att is not None else 0,
        "per_target": lag, "micro_batches": max(1, batch // mbs), "audit_micro_k": c.get("audit_micro_k", 1),
        "audit_summary": eng.audit_summary(),
        "clean_nodes_blamed": clean_blamed,
        "clean_nodes_compromised": [n for n in compromised if n not in c["targets"]],
        "clean_nodes_resharded": sorted({n for r in rs for n in r["from_nodes"] if n not in c["targets"]}),
        "ms_per_step": round(1000 * wall / max(1, steps), 2),
        "reshards": [{"step": r["step"], "from_nodes": r["from_nodes"], "to_nodes": r["to_nodes"],
                      "migration_ms": round(1000 * r["migration_time"], 2),
                      "estimated_ms": round(1000 * r["estimated_migration_time"], 2),
                      "phases_ms": {k: round(1000 * v, 2) for k, v in r.get("phases", {}).items() if k.endswith("_s")},
                      "rebuild_new_reserved_mb": round(r.get("phases", {}).get("rebuild_new_reserved_bytes", 0) / 2**20, 1),
                      "moved_params": r["moved_params"], "restored_from_shadow": r.get("restored_from_shadow"),
                      "restored_from_initial": r.get("restored_from_initial"),
                      "plan": r["plan"]} for r in rs],
        "plan_before": plan0, "plan_after": eng.plan.describe(), "num_stages_after": eng.plan.num_stages,
        "final_trust": [round(eng.trust.get_trust_score(n), 3) for n in range(8)],
        "final_status": [eng.trust.get_node_status(n).value for n in range(8)],
        "loss_curve": losses, "wall_s": round(wall, 1),
        # every per-stage verdict: (step, node, kind, ground truth, output z, gradient z)
        "events": [(r["step"], r["node_id"], r.get("attack_type"), bool(r.get("ground_truth")),
                    round(float(r.get("output_stats", {}).get("z", 0.0)), 2),
                    round(float(r.get("gradient_stats", {}).get("z", 0.0)), 2)) for r in eng.attack_history],
    }
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="3,4,5", help="comma list of 3, 4, 5, clean, 3s, dx, last, 3m, 3ms, 5m, liar, 3a, 3am")
    ap.add_argument("--seeds", default="3", help="comma list of attacker / monitor seeds")
    ap.add_argument("--no-reassign", action="store_true", help="detection only: the target keeps its layers, so "
                    "every injection is scored (a re-shard ends the attack after the first detections)")
    ap.add_argument("--no-audit", action="store_true")
    ap.add_argument("--device", default="cuda:0" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--start", type=int, default=100)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--mbs", type=int, default=2)
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--p-attack", type=float, default=0.3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--small", action="store_true", help="tiny models (CPU smoke of the same flow)")
    ap.add_argument("--detector-warmup", type=int, default=50)
    args = ap.parse_args()
    for cid in [int(x) if x.isdigit() else x for x in args.configs.split(",")]:
        for seed in [int(x) for x in args.seeds.split(",")]:
            rec = run(cid, args.device, args.steps, args.start, args.batch, args.mbs, args.seq_len, args.p_attack,
                      args.small, args.detector_warmup, seed=seed, reassign=not args.no_reassign,
                      audit=not args.no_audit)
            line = json.dumps(rec)
            print(line, flush=True)
            if args.out:
                with open(args.out, "a") as f:
                    f.write(line + "\n")
            if args.device.startswith("cuda"):
                torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
