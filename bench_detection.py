#!/usr/bin/env python3
"""Attack-detection benchmark: precision / recall / F1 (the second half of the BASELINE metric).

Part ``protocol`` replays the measurement protocol of BASELINE.md's "reference-behaviour" table
(the reference's ``detect_gradient_poisoning``, attack_detector.py:109-141): 100 clean warm-up
steps, then 200 steps where each step is attacked with p = 0.2; gradients are 4 tensors
[256, 256] drawn from N(0, 0.01), seed 0.  Three detectors see identical streams:

* ``reference``  — AttackDetector(compat=True): the reference's decision rule, bugs included
                   (current sample inside its own baseline; cross-tensor cosine);
* ``detector``   — AttackDetector() defaults: baseline excludes the current sample, flagged
                   samples quarantined, EMA-reference cosine;
* ``engine``     — the engine's device z-score (DeviceZScore: median / 1.4826*MAD over a
                   100-step window, exclude-current, quarantine) on the same statistic vector;
                   the HIP kernel when ``--device cuda``.

Part ``engine`` trains a GPT-2 through the PipelineEngine (local multi-stage mode: every
stage on one device) with the AdversarialAttacker poisoning one stage on a random 20 % of the
steps after a clean warm-up, and scores the engine's own per-stage, per-step verdicts against
the attacker's ground truth (gradient poisoning x10 / x3 / noise / zero / sign-flip, parameter
perturbation, Byzantine activation tampering).

    python bench_detection.py --part protocol
    python bench_detection.py --part engine --device cuda:0 --model gpt2-medium --stages 8
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

PROTOCOL_ATTACKS = {
    "scale_x10": lambda g, r: [t * 10.0 for t in g],
    "scale_x3": lambda g, r: [t * 3.0 for t in g],
    "scale_x1.5": lambda g, r: [t * 1.5 for t in g],
    "noise_sigma_x1": lambda g, r: [t + torch.randn(t.shape, generator=r) * 0.01 for t in g],
    "noise_sigma_x5": lambda g, r: [t + torch.randn(t.shape, generator=r) * 0.05 for t in g],
    "sign_flip": lambda g, r: [-t for t in g],
    "zero": lambda g, r: [torch.zeros_like(t) for t in g],
}
# reference numbers measured during the survey (same protocol)
REFERENCE_F1 = {"scale_x10": 0.702, "scale_x3": 0.604, "scale_x1.5": 0.426, "noise_sigma_x1": 0.490,
                "noise_sigma_x5": 0.702, "sign_flip": 0.0, "zero": 0.520}


def _prf(tp, fp, fn):
    p = tp / (tp + fp) if tp + fp else 0.0
    r = tp / (tp + fn) if tp + fn else 0.0
    return {"tp": tp, "fp": fp, "fn": fn, "precision": round(p, 3), "recall": round(r, 3),
            "f1": round(2 * p * r / (p + r), 3) if p + r else 0.0}


def run_protocol(device: str, warm: int = 100, steps: int = 200, p_attack: float = 0.2, seed: int = 0):
    from trustworthy_dl.ops.stats import DeviceZScore
    from trustworthy_dl.security.attack_detection import GRAD_STATS, AttackDetector, gradient_statistics

    results = {}
    for name, attack in PROTOCOL_ATTACKS.items():
        g = torch.Generator().manual_seed(seed)
        dets = {"reference": AttackDetector(compat=True), "detector": AttackDetector()}
        eng = DeviceZScore(len(GRAD_STATS), device)
        ema_ref = None
        counts = {k: [0, 0, 0] for k in ("reference", "detector", "engine")}
        for step in range(warm + steps):
            grads = [torch.randn(256, 256, generator=g) * 0.01 for _ in range(4)]
            attacked = step >= warm and float(torch.rand(1, generator=g)) < p_attack
            if attacked:
                grads = attack(grads, g)
            for k, d in dets.items():
                flag = d.detect_gradient_poisoning(grads, 0, step)
                _count(counts[k], flag, attacked, step >= warm)
            # engine: same statistic vector (EMA-reference cosine), device z-score decision
            st = gradient_statistics(grads, ema_ref, "reference")
            vec = torch.tensor([st[n] for n in GRAD_STATS], dtype=torch.float32, device=device)
            flag = bool(eng.observe(vec)[0].item() > 0)
            _count(counts["engine"], flag, attacked, step >= warm)
            if not (flag and step >= warm):  # the engine only folds accepted gradients into its reference
                ema_ref = [t.clone() for t in grads] if ema_ref is None else \
                    [0.9 * r + 0.1 * t for r, t in zip(ema_ref, grads)]
        results[name] = {k: _prf(*v) for k, v in counts.items()}
        results[name]["reference_published_survey_f1"] = REFERENCE_F1[name]
    return results


def _count(c, flag, attacked, scored):
    if not scored:
        return
    if flag and attacked:
        c[0] += 1
    elif flag:
        c[1] += 1
    elif attacked:
        c[2] += 1


ENGINE_SCENARIOS = {
    "grad_scale_x10": dict(attack_types=["gradient_poisoning"], gradient_mode="scale", gradient_scale=10.0),
    "grad_scale_x3": dict(attack_types=["gradient_poisoning"], gradient_mode="scale", gradient_scale=3.0),
    "grad_noise": dict(attack_types=["gradient_poisoning"], gradient_mode="noise", intensity=0.5),
    "grad_zero": dict(attack_types=["gradient_poisoning"], gradient_mode="zero"),
    "grad_sign_flip": dict(attack_types=["gradient_poisoning"], gradient_mode="sign_flip"),
    "param_perturb": dict(attack_types=["model_poisoning"], intensity=0.05),
    "byzantine_output": dict(attack_types=["byzantine"], intensity=0.5),
}


DATA_VOCAB = [0]
WARMUP = [0]       # linear lr warm-up steps   # > 0: the Markov stream uses only this many token ids (learnable in a few hundred steps)


def _batches(data: str, batch: int, seq_len: int, vocab: int, n: int, seed: int = 0):
    """Training batches: ``random`` uniform tokens (flat loss, stationary gradients) or ``markov``
    (a learnable order-1 Markov stream: the loss falls and gradients drift / correlate)."""
    if data == "markov":
        from trustworthy_dl.utils.data_loader import MarkovLanguageModeling
        yield from MarkovLanguageModeling(batch, seq_len, DATA_VOCAB[0] or vocab, num_batches=n, seed=seed)
        return
    g = torch.Generator().manual_seed(seed)
    for _ in range(n):
        ids = torch.randint(0, vocab, (batch, seq_len + 1), generator=g)
        yield {"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()}


def _engine(device, model_name, stages, batch, mbs, seq_len, vocab, lr, attacker=None, robust="detrend",
            reassign=False):
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.flat import AdamWConfig
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    from trustworthy_dl.utils.metrics import MetricsCollector
    extra = {"vocab_size": vocab} if vocab != 50257 else {}
    model = get_model(model_name, seq_len=seq_len, seed=11, **extra)
    cfg = EngineConfig(num_nodes=stages, micro_batches=max(1, batch // mbs), seq_len=seq_len, device=device,
                       adamw=AdamWConfig(lr=lr, weight_decay=0.01, max_grad_norm=1.0, warmup_steps=WARMUP[0]),
                       attack_detection=True, gradient_verification=True, quarantine=True, reassign=reassign,
                       verifier={"robust_baseline": robust})
    return PipelineEngine(model, cfg, attacker=attacker, metrics=MetricsCollector())


def run_fp(device: str, model_name: str, stages: int, steps: int, warm: int, batch: int, mbs: int, seq_len: int,
           vocab: int, data: str, lr: float, robust: str):
    """False-positive rate of the engine's verdicts on CLEAN training (no attacker): flagged
    (stage, step) pairs after the warm-up / all scored pairs, plus the loss curve."""
    eng = _engine(device, model_name, stages, batch, mbs, seq_len, vocab, lr, robust=robust)
    t0 = time.perf_counter()
    for b in _batches(data, batch, seq_len, vocab, warm + steps):
        eng.train_step(b)
    eng.flush()
    flags = [(a["step"], a["node_id"], a["attack_type"]) for a in eng.attack_history if a["step"] > warm]
    losses = [m["loss"] for m in eng.metrics.batch_metrics if m.get("loss") is not None]
    pairs = steps * stages
    res = {"data": data, "data_vocab": DATA_VOCAB[0] or vocab, "lr": lr, "lr_warmup": WARMUP[0], "robust": robust,
           "steps_scored": steps, "stages": stages, "false_positives": len(flags),
           "fp_rate": round(len(flags) / pairs, 5), "flags": flags[:20],
           "loss_first": round(losses[0], 4), "loss_at_warm": round(losses[warm - 1], 4), "loss_last": round(losses[-1], 4),
           "loss_curve_every_25": [round(x, 4) for x in losses[::25]],
           "final_trust": [round(eng.trust.get_trust_score(n), 3) for n in range(stages)],
           "wall_s": round(time.perf_counter() - t0, 1)}
    print(json.dumps({"fp": res}), flush=True)
    return res


def run_engine(device: str, model_name: str, stages: int, steps: int, warm: int, batch: int, mbs: int,
               seq_len: int, scenarios, target: int, p_attack: float, vocab: int = 50257, data: str = "random",
               lr: float = 1e-4, robust: str = "detrend"):
    from trustworthy_dl.attacks.adversarial_attacks import AdversarialAttacker, AttackConfig
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.flat import AdamWConfig
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine

    out = {}
    for name in scenarios:
        kw = dict(ENGINE_SCENARIOS[name])
        attacker = AdversarialAttacker(AttackConfig(target_nodes=[target], start_step=warm, probability=p_attack,
                                                    seed=7, **kw))
        attacker.activate_attacks()
        eng = _engine(device, model_name, stages, batch, mbs, seq_len, vocab, lr, attacker=attacker, robust=robust)
        t0 = time.perf_counter()
        for b in _batches(data, batch, seq_len, vocab, warm + steps):
            eng.train_step(b)
        eng.flush()
        m = attacker.detection_metrics()
        out[name] = {"tp": m["tp"], "fp": m["fp"], "fn": m["fn"], "precision": round(m["precision"], 3),
                     "recall": round(m["recall"], 3), "f1": round(m["f1"], 3),
                     "mean_time_to_detect_steps": m["mean_time_to_detect_steps"],
                     "injections": len(attacker.injections), "final_loss": eng.last_loss,
                     "final_trust": [round(eng.trust.get_trust_score(n), 3) for n in range(stages)],
                     "target_status": eng.trust.get_node_status(target).value,
                     "wall_s": round(time.perf_counter() - t0, 1)}
        print(json.dumps({name: out[name]}), flush=True)
        del eng
        if device.startswith("cuda"):
            torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--part", choices=["protocol", "engine", "fp", "all"], default="protocol")
    ap.add_argument("--data", choices=["random", "markov"], default="markov")
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--robust", default="detrend", help="engine z-score baseline: detrend | 1 (median/MAD) | 0")
    ap.add_argument("--data-vocab", type=int, default=0, help="Markov stream over this many token ids (0 = all)")
    ap.add_argument("--lr-warmup", type=int, default=0)
    ap.add_argument("--device", default="cuda:0" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--model", default=None)
    ap.add_argument("--stages", type=int, default=None)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warm", type=int, default=100)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--mbs", type=int, default=None)
    ap.add_argument("--seq-len", type=int, default=None)
    ap.add_argument("--target", type=int, default=None)
    ap.add_argument("--vocab", type=int, default=None)
    ap.add_argument("--p-attack", type=float, default=0.2)
    ap.add_argument("--scenarios", default=",".join(ENGINE_SCENARIOS))
    ap.add_argument("--out", default=None, help="write the JSON result here too")
    args = ap.parse_args()
    gpu = args.device.startswith("cuda")
    res = {"device": args.device}
    if args.part in ("protocol", "all"):
        res["protocol"] = run_protocol(args.device)
        print(json.dumps({"protocol": res["protocol"]}), flush=True)
    robust = args.robust if args.robust == "detrend" else int(args.robust)
    DATA_VOCAB[0] = args.data_vocab
    WARMUP[0] = args.lr_warmup
    if args.part in ("fp", "all"):
        model = args.model or ("gpt2-medium" if gpu else "gpt2-tiny")
        stages = args.stages or (8 if gpu else 4)
        res["fp"] = run_fp(args.device, model, stages, args.steps, args.warm, args.batch or (8 if gpu else 4),
                           args.mbs or (4 if gpu else 2), args.seq_len or (1024 if gpu else 64),
                           args.vocab or (50257 if gpu else 1024), args.data, args.lr, robust)
    if args.part in ("engine", "all"):
        model = args.model or ("gpt2-medium" if gpu else "gpt2-tiny")
        stages = args.stages or (8 if gpu else 4)
        res["engine"] = run_engine(args.device, model, stages, args.steps, args.warm,
                                   args.batch or (8 if gpu else 4), args.mbs or (4 if gpu else 2),
                                   args.seq_len or (1024 if gpu else 64), args.scenarios.split(","),
                                   args.target if args.target is not None else stages // 2, args.p_attack,
                                   args.vocab or (50257 if gpu else 1024), args.data, args.lr, robust)
        res["engine_config"] = {"model": model, "stages": stages, "steps": args.steps, "warm": args.warm,
                                "p_attack": args.p_attack, "data": args.data, "lr": args.lr, "robust": str(robust),
                                "data_vocab": args.data_vocab, "lr_warmup": args.lr_warmup}
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
