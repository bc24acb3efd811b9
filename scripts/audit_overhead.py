#!/usr/bin/env python3
"""Cost of the audit protocol on one GPU: GPT-2-medium, 8 pipeline stages in local mode (every
stage on this GPU, so every stage is also audited here), M = 16 micro-batches, T = 1024, bf16.

Variants, interleaved per round on the same box: ``off`` (no audit), ``fwd`` (forward recompute
audit only), ``mirror`` (the full protocol: contribution ring + BLAKE2s Merkle commitments + keyed
sketches + k opened micro-batches recomputed + live optimizer mirrors).  One JSON line per
(variant, round): ms/step, and for ``mirror`` the protocol's own accounting (audit_summary: device
ms of the audit phase, bytes it would ship between ranks, device memory of rings + mirrors).

    python scripts/audit_overhead.py --steps 6 --warmup 2 --rounds 2 --out gpurun_out/r6_audit_overhead.jsonl
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from trustworthy_dl.runtime.hwqueues import ensure_hw_queues  # noqa: E402
ensure_hw_queues()
from trustworthy_dl.models import get_model  # noqa: E402
from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine  # noqa: E402


def run(variant, args):
    m = get_model(args.model, seq_len=args.seq, seed=1)
    cfg = dict(num_nodes=args.stages, micro_batches=args.micro, device="cuda:0", seq_len=args.seq, monitor_seed=0,
               reassign=False, audit_micro_k=args.k, audit_targeted=False)
    if variant == "off":
        cfg["audit"] = False
    elif variant == "fwd":
        cfg["audit_backward"] = False
    eng = PipelineEngine(m, EngineConfig(**cfg))
    g = torch.Generator().manual_seed(0)
    batches = []
    for _ in range(2):
        ids = torch.randint(0, 50257, (args.batch, args.seq + 1), generator=g)
        batches.append({"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()})
    for i in range(args.warmup):
        eng.train_step(batches[i % 2])
    torch.cuda.synchronize()
    prof = None
    if args.cprofile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    for i in range(args.steps):
        eng.train_step(batches[i % 2])
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / args.steps
    if prof is not None:
        prof.disable()
        import io
        import pstats
        buf = io.StringIO()
        pstats.Stats(prof, stream=buf).sort_stats("cumulative").print_stats(45)
        with open(f"{args.cprofile}.{variant}.txt", "w") as f:
            f.write(buf.getvalue())
    eng.flush()
    rec = {"variant": variant, "ms_per_step": round(ms, 2), "tokens_per_s": round(args.batch * args.seq / ms * 1e3, 1),
           "model": args.model, "stages": args.stages, "micro_batches": args.micro, "batch": args.batch,
           "seq": args.seq, "audit_micro_k": args.k, "blamed": len(eng.attack_history)}
    if variant != "off":
        rec["audit"] = eng.audit_summary()
    del eng
    torch.cuda.empty_cache()
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-medium")
    ap.add_argument("--stages", type=int, default=8)
    ap.add_argument("--micro", type=int, default=16)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--k", type=int, default=1)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--variants", default="off,fwd,mirror")
    ap.add_argument("--out", default="gpurun_out/r6_audit_overhead.jsonl")
    ap.add_argument("--round-id", type=int, default=0)
    ap.add_argument("--cprofile", default="", help="write a host cProfile of the timed steps to <path>.<variant>.txt")
    ap.add_argument("--inproc", action="store_true", help="run in this process (default: one process per run)")
    args = ap.parse_args()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    variants = args.variants.split(",")
    if not args.inproc and (len(variants) > 1 or args.rounds > 1):
        # every (round, variant) in a fresh process: engines of 35 GB of rings + mirrors do not share
        # one allocator's fragmentation, and no run inherits another's warm caches
        import subprocess
        for r in range(args.rounds):
            for v in variants:
                cmd = [sys.executable, os.path.abspath(__file__), "--inproc", "--variants", v, "--rounds", "1",
                       "--round-id", str(r), "--model", args.model, "--stages", str(args.stages),
                       "--micro", str(args.micro), "--batch", str(args.batch), "--seq", str(args.seq),
                       "--k", str(args.k), "--steps", str(args.steps), "--warmup", str(args.warmup), "--out", args.out]
                rc = subprocess.run(cmd).returncode
                if rc != 0:
                    sys.exit(rc)
        return
    with open(args.out, "a") as f:
        for v in variants:
            rec = run(v, args)
            rec["round"] = args.round_id
            print(json.dumps(rec), flush=True)
            f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
