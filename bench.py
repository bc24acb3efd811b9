#!/usr/bin/env python3
"""Headline benchmark: GPT-2-medium pipeline-model-parallel training with gradient verification on.

Metric (BASELINE.json): tokens/sec, GPT-2-medium, MP = number of GPUs (pp1/2/4/8), trust +
gradient verification + output anomaly detection active in every step, bf16 compute with fp32
master weights + fused AdamW, synthetic token data, random-init weights.

    python bench.py                       # N=1 defaults
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P \\
        bench.py --gpus N --steps K --warmup W

Weak scaling: the global batch is ``--batch-per-gpu`` (default 64 sequences of 1024 tokens) times
N, split into micro-batches of ``--mbs`` sequences; each stage does 1/N of the layers for N times
the tokens, so per-GPU work is fixed.  At N=8 the global batch is 512 x 1024 tokens, GPT-2's own
training batch; 1F1B keeps at most S micro-batches in flight per stage, so the larger batch costs
no extra activation memory, while the pipeline fill/drain and the per-step optimizer and
verification passes are spread over twice the tokens of the README's 32 (measured on one MI355X:
337k tok/s at 32 sequences, 349k at 64; ``--batch-per-gpu 32`` reproduces the former).  Timing: W untimed steps,
then barrier + device sync, K timed optimizer steps, barrier + device sync; the MAX elapsed over
ranks is reported.  ``value`` = whole-job tokens/s.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# before the first GPU call (torch.cuda.is_available() below starts the HIP runtime): RCCL streams
# on hardware queues of their own, so pre-posted receives never block compute (runtime/hwqueues.py)
from trustworthy_dl.runtime.hwqueues import ensure_hw_queues, effective_hw_queues  # noqa: E402
ensure_hw_queues()


# Single-GPU GPT-2-medium throughput (k tokens/s) per micro-batch size, from per-unit fwd+bwd
# timings on MI355X (scripts/time_units.py at micro-batch 4/8/16/32: 24 blocks + LM head +
# embedding per sequence; profiles/r1_gpt2m_unit_times.jsonl): larger micro-batches feed the GEMMs
# and the attention kernels larger tiles.  Used only to choose the micro-batch size.
_MBS_EFF = {4: 220.9, 8: 269.8, 16: 329.3, 32: 354.8}
# fill/drain slot cost relative to a steady-state slot: with the B/W split the drain advances one
# stage per (F + B_input) ~ 2/3 of a full (F + B_input + W) slot
_BUBBLE_WEIGHT = 2.0 / 3.0


def choose_mbs(global_batch: int, stages: int) -> int:
    """1F1B step time ~ (M + w (S - 1)) micro-batch slots of mbs / eff(mbs) each (M = batch / mbs):
    few big micro-batches run efficient kernels but leave a long fill/drain bubble."""
    best, best_t = None, float("inf")
    for mbs, eff in _MBS_EFF.items():
        if global_batch % mbs:
            continue
        m = global_batch // mbs
        if m < stages and stages > 1:
            continue
        t = (m + _BUBBLE_WEIGHT * (stages - 1)) * mbs / eff
        if t < best_t:
            best, best_t = mbs, t
    return best or 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="gpt2-medium")
    ap.add_argument("--seq-len", type=int, default=1024)
    ap.add_argument("--batch-per-gpu", type=int, default=64)
    ap.add_argument("--mbs", default="auto",
                    help="sequences per micro-batch, or 'auto' (pipeline-bubble vs GEMM-efficiency model)")
    ap.add_argument("--no-verify", action="store_true", help="disable detection/verification (ablation)")
    ap.add_argument("--lr", type=float, default=5e-5)
    ap.add_argument("--dp", type=int, default=1,
                    help="data-parallel pipeline replicas (default 1: the headline is MP = N stages)")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--trace-phases", default="",
                    help="write a per-phase HIP-event breakdown (JSON, + Chrome trace next to it) to this path")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print(f"--gpus {args.gpus} needs torch.distributed.run --nproc-per-node {args.gpus}", file=sys.stderr)
            sys.exit(2)
    use_cuda = torch.cuda.is_available()
    if use_cuda:
        torch.cuda.set_device(local_rank)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend="nccl" if use_cuda else "gloo",
                                device_id=torch.device("cuda", local_rank) if use_cuda else None)

    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.flat import AdamWConfig
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine

    N = world
    dp = max(1, args.dp)
    stages = N // dp
    global_batch = args.batch_per_gpu * N
    per_replica = global_batch // dp
    mbs = choose_mbs(per_replica, stages) if args.mbs == "auto" else int(args.mbs)
    M = per_replica // mbs
    model = get_model(args.model, seq_len=args.seq_len, seed=1234)
    verify = not args.no_verify
    cfg = EngineConfig(num_nodes=N, micro_batches=M, seq_len=args.seq_len, data_parallel=dp,
                       adamw=AdamWConfig(lr=args.lr, weight_decay=0.01, max_grad_norm=1.0),
                       attack_detection=verify, gradient_verification=verify, quarantine=verify,
                       reassign=False, trace_phases=bool(args.trace_phases))
    engine = PipelineEngine(model, cfg)
    del model

    g = torch.Generator().manual_seed(0)
    V = 50257
    batches = []
    for _ in range(2):
        ids = torch.randint(0, V, (global_batch, args.seq_len + 1), generator=g)
        batches.append({"input": ids[:, :-1].contiguous().pin_memory() if use_cuda else ids[:, :-1].contiguous(),
                        "target": ids[:, 1:].contiguous().pin_memory() if use_cuda else ids[:, 1:].contiguous()})

    def sync():
        if world > 1:
            dist.barrier()
        if use_cuda:
            torch.cuda.synchronize()

    for i in range(args.warmup):
        engine.train_step(batches[i % 2])
    engine.flush()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        engine.train_step(batches[i % 2])
    sync()
    elapsed = time.perf_counter() - t0
    engine.flush()
    el = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}" if use_cuda else "cpu")
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el)
    tokens = global_batch * args.seq_len * args.steps
    tps = tokens / elapsed
    if rank == 0:
        line = {
            "metric": "tokens/sec GPT-2-medium MP=N with grad-verify on",
            "value": round(tps, 1), "unit": "tokens/s", "n_gpus": N, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16", "data": "synthetic tokens, random-init weights",
            "config": {"model": args.model, "global_batch": global_batch, "seq_len": args.seq_len,
                       "micro_batch": mbs, "micro_batches": M,
                       "parallelism": f"pp{stages}" + (f"xdp{dp}" if dp > 1 else ""),
                       "grad_verify": verify, "output_detection": verify, "trust_update": True,
                       "plan": engine.plan.describe(), "last_loss": engine.last_loss,
                       "p2p_mode": engine.p2p_mode, "hw_queues": effective_hw_queues()},
        }
        print(json.dumps(line), flush=True)
    if args.trace_phases:
        engine.tracer.resolve(block=True)
        base, ext = os.path.splitext(args.trace_phases)
        path = f"{base}_rank{rank}{ext or '.json'}"
        with open(path, "w") as f:
            json.dump({"rank": rank, "stage_plan": engine.plan.describe(),
                       "ms_per_step": engine.tracer.summary(skip=args.warmup)}, f, indent=1)
        engine.tracer.export_chrome_trace(f"{base}_rank{rank}.trace.json", pid=rank)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
