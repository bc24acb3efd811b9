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

Failure reporting (multi-rank): every rank publishes where it is (runtime/progress.py) to the
c10d store; when a rank raises, or any rank stops advancing for ``--watchdog`` seconds, rank 0
prints ONE failure JSON line (``value`` null, ``error``, ``failed_phase`` per rank) and the job
exits non-zero.  ``--debug-fault hang|raise --debug-fault-rank R --debug-fault-step S`` injects
such a failure (tests/test_bench_gloo.py).
"""
from __future__ import annotations

import argparse
import datetime
import json
import os
import sys
import time
import traceback

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
# 64 (one micro-batch: N=1 only in practice): +2.1 % over 32 in an interleaved A/B with the LM head
# unchunked (profiles/r2_mbs64_ab.txt)
_MBS_EFF = {4: 220.9, 8: 269.8, 16: 329.3, 32: 354.8, 64: 362.3}
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
    ap.add_argument("--no-verify", action="store_true",
                    help="ablation: no output / gradient statistics, quantiles, z-scores or weight checksums "
                         "(only a bare sum-of-squares pass for gradient clipping)")
    ap.add_argument("--lr", type=float, default=5e-5)
    ap.add_argument("--dp", type=int, default=1,
                    help="data-parallel pipeline replicas (default 1: the headline is MP = N stages)")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--trace-phases", default="",
                    help="write a per-phase HIP-event breakdown (JSON, + Chrome trace next to it) to this path")
    ap.add_argument("--p2p-mode", default="auto", choices=["auto", "async", "grouped"],
                    help="pipeline P2P: pre-posted receives on per-direction communicators (async) or one "
                         "batched exchange per transfer (grouped); auto = async when the HIP runtime has "
                         "enough hardware queues")
    ap.add_argument("--timeout", type=float, default=600.0,
                    help="process-group timeout (s) for init and collectives")
    ap.add_argument("--watchdog", type=float, default=300.0,
                    help="seconds without progress on any rank before the run is reported failed (0 = off)")
    ap.add_argument("--reassign-at", type=int, default=-1,
                    help="after this many steps (warmup included), exclude the last pipeline rank and "
                         "re-shard its layers over the others (exercises migration mid-run)")
    ap.add_argument("--audit-targeted", action="store_true",
                    help="audit the anomaly-picked micro-batch too (EngineConfig.audit_targeted; one host "
                         "read per step on the auditors)")
    ap.add_argument("--debug-fault", default="", choices=["", "hang", "raise"])
    ap.add_argument("--debug-fault-rank", type=int, default=-1)
    ap.add_argument("--debug-fault-step", type=int, default=1)
    args = ap.parse_args()
    try:
        run(args)
    except SystemExit:
        raise
    except BaseException as e:  # noqa: BLE001 - every failure becomes a legible line + non-zero exit
        _fail(args, "error", f"{type(e).__name__}: {e}\n{traceback.format_exc()}")


_WATCHDOG = None
METRIC = "tokens/sec GPT-2-medium MP=N with grad-verify on"   # the BASELINE.json headline (defaults)


def _metric(args) -> str:
    """The headline name for the default run; other models / --no-verify say what they measured."""
    if args.model == "gpt2-medium" and not args.no_verify:
        return METRIC
    name = {"gpt2-small": "GPT-2-small", "gpt2-medium": "GPT-2-medium", "gpt2-large": "GPT-2-large",
            "gpt2-xl": "GPT-2-xl"}.get(args.model, args.model)
    return f"tokens/sec {name} MP=N with grad-verify {'off' if args.no_verify else 'on'}"


def _failure_line(args, kind: str, marks, errors) -> str:
    from trustworthy_dl.runtime import progress
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if errors:
        msg = "; ".join(f"rank {e['rank']} raised in '{e['phase']}': {e['error'].splitlines()[0]}" for e in errors)
    elif kind == "stall":
        stale = sorted(marks.items(), key=lambda kv: -(kv[1].get("stalled_s") or 0))
        r, st = stale[0]
        msg = f"no progress for {st.get('stalled_s')}s on rank {r} in '{st.get('phase')}'"
    else:
        msg = kind
    return json.dumps({
        "metric": _metric(args), "value": None, "unit": "tokens/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": None, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic tokens, random-init weights",
        "error": msg, "failure_kind": kind,
        "failed_phase": {str(r): m.get("phase") for r, m in marks.items()},
        "stalled_s": {str(r): m.get("stalled_s") for r, m in marks.items()},
        "errors": errors, "config": {"model": args.model, "p2p_mode": args.p2p_mode},
        "phase_now": progress.current()["phase"]})


def _fail(args, kind: str, message: str):
    """This rank's main loop raised: rank 0 prints the failure line, other ranks hand the error
    to rank 0 through the store (and print it to stderr); exit non-zero either way."""
    from trustworthy_dl.runtime import progress
    rank = int(os.environ.get("RANK", "0"))
    print(f"[bench] rank {rank} failed in '{progress.current()['phase']}': {message}", file=sys.stderr, flush=True)
    if _WATCHDOG is not None:
        _WATCHDOG.report_error(message)          # rank 0: prints the line and exits here
    elif rank == 0:
        rec = [{"rank": 0, "phase": progress.current()["phase"], "error": message[-2000:]}]
        print(_failure_line(args, kind, {0: progress.current()}, rec), flush=True)
    sys.stdout.flush()
    os._exit(1)


def run(args):
    global _WATCHDOG
    from trustworthy_dl.runtime import progress

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
    progress.mark("init_process_group")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend="nccl" if use_cuda else "gloo",
                                timeout=datetime.timedelta(seconds=args.timeout),
                                device_id=torch.device("cuda", local_rank) if use_cuda else None)
        _WATCHDOG = progress.StallWatchdog(
            rank, world, args.watchdog, store=dist.distributed_c10d._get_default_store(),
            on_failure=lambda kind, marks, errs: print(_failure_line(args, kind, marks, errs), flush=True)
            if rank == 0 else None).start()
    # TDL_COMMCHECK=<dir>: record this rank's communication for the RCCL-model replay
    # (trustworthy_dl/runtime/commcheck.py; the multi-rank CPU tests check the schedule with it)
    from trustworthy_dl.runtime import commcheck
    _rec = commcheck.maybe_install() if world > 1 else None
    hwq = effective_hw_queues()
    print(f"[bench] rank {rank} local_rank {local_rank} GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES')} "
          f"effective_hw_queues={hwq}", file=sys.stderr, flush=True)

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
    progress.mark("build engine")
    p2p = {"auto": "async"}.get(args.p2p_mode, args.p2p_mode)
    cfg = EngineConfig(p2p_mode=p2p, num_nodes=N, micro_batches=M, seq_len=args.seq_len, data_parallel=dp,
                       adamw=AdamWConfig(lr=args.lr, weight_decay=0.01, max_grad_norm=1.0),
                       attack_detection=verify, gradient_verification=verify, quarantine=verify,
                       param_integrity=verify,
                       reassign=False, trace_phases=bool(args.trace_phases),
                       audit_targeted=True if args.audit_targeted else None)
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
        commcheck.note_host_sync(device=True)
        if use_cuda:
            torch.cuda.synchronize()

    # the next batch's host->device copy runs on a copy stream under the current step
    # (utils/prefetch.py); each rank copies only what its stages consume
    from trustworthy_dl.utils.prefetch import DevicePrefetcher
    keys = None
    if engine.distributed:
        st = engine.my_stage()
        keys = ([] if st is None else (["input"] if st.stage_id == 0 else []) + (["target"] if st.computes_loss else []))
    seq = (batches[i % 2] for i in range(args.warmup + args.steps))
    feed = iter(seq) if os.environ.get("TDL_BENCH_PREFETCH", "1") == "0" else \
        DevicePrefetcher(seq, engine.device, keys=keys)   # (=0: the engine's own copies, A/B)
    done = [0]

    def step(i):
        if args.debug_fault and rank == args.debug_fault_rank and done[0] == args.debug_fault_step:
            progress.mark(f"step {done[0] + 1}: injected {args.debug_fault} (--debug-fault)")
            if args.debug_fault == "raise":
                raise RuntimeError("injected fault (--debug-fault raise)")
            while True:                      # a rank that stops answering (its peers block in P2P)
                time.sleep(3600)
        engine.train_step(next(feed))
        done[0] += 1
        if done[0] == args.reassign_at:
            progress.mark(f"step {done[0]}: re-shard away from rank {engine.plan.ranks[-1]}")
            engine.flush()
            engine.reassign([engine.plan.ranks[-1]], done[0])

    for i in range(args.warmup):
        step(i)
    engine.flush()
    progress.mark("timing barrier (start)")
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    progress.mark("timing barrier (end)")
    sync()
    elapsed = time.perf_counter() - t0
    engine.flush()
    progress.mark("report")
    el = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}" if use_cuda else "cpu")
    hwq_all = [hwq]
    inv = engine.comm_inventory()
    inv["audit"] = engine.audit_summary()
    inv_all = [inv]
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        hwq_all = [None] * world
        dist.all_gather_object(hwq_all, hwq)
        inv_all = [None] * world
        dist.all_gather_object(inv_all, inv)
    if use_cuda and not all(i["within_queue_budget"] for i in inv_all):
        print(f"[bench] WARNING: a rank's HIP streams exceed its hardware queues: {inv_all}", file=sys.stderr, flush=True)
    elapsed = float(el)
    tokens = global_batch * args.seq_len * args.steps
    tps = tokens / elapsed
    if rank == 0:
        from trustworthy_dl.ops import gemm as gemm_mod
        line = {
            "metric": _metric(args),
            "value": round(tps, 1), "unit": "tokens/s", "n_gpus": N, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16", "data": "synthetic tokens, random-init weights",
            "config": {"model": args.model, "global_batch": global_batch, "seq_len": args.seq_len,
                       "micro_batch": mbs, "micro_batches": M,
                       "parallelism": f"pp{stages}" + (f"xdp{dp}" if dp > 1 else ""),
                       "grad_verify": verify, "output_detection": verify, "trust_update": True,
                       # deterministic stage cross-check (recompute audit; needs >= 2 stages)
                       "stage_audit": bool(engine.cfg.audit and engine.plan.num_stages > 1),
                       "plan": engine.plan.describe(), "last_loss": engine.last_loss,
                       "detections": len(engine.attack_history),
                       "flagged": sorted({(a["step"], a["node_id"], a["attack_type"]) for a in engine.attack_history})[:8],
                       "p2p_mode": engine.p2p_mode, "p2p_mode_requested": args.p2p_mode,
                       "native_gemm": "fc fwd+gelu (pd), proj dgrad+dgelu (pp), LM-head dX (pd), all weight gradients "
                                      f"({gemm_mod.WGRAD_KERNEL}"
                                      + (", qkv+o and fc+proj grouped" if gemm_mod.WGRAD_GROUPED and gemm_mod.WGRAD_KERNEL == "pd"
                                         and os.environ.get("TDL_WGRAD_GROUPED_MLP", "1") != "0" else "")
                                      + (", qkv+o grouped" if gemm_mod.WGRAD_GROUPED and gemm_mod.WGRAD_KERNEL == "pd"
                                         and os.environ.get("TDL_WGRAD_GROUPED_MLP", "1") == "0" else "") + ")",
                       "native_wgrad": gemm_mod.WGRAD_KERNEL,
                       "hw_queues": hwq, "hw_queues_per_rank": hwq_all,
                       # per-rank RCCL communicators / HIP streams (compute + verification + one per
                       # communicator) vs the hardware-queue budget (PipelineEngine.comm_inventory)
                       "rccl_comms_per_rank": [i["rccl_comms"] for i in inv_all],
                       "hip_streams_per_rank": [i["hip_streams"] for i in inv_all],
                       "process_groups_created": inv["groups_created"],
                       "within_queue_budget": all(i["within_queue_budget"] for i in inv_all),
                       # recompute audit (forward + backward) per rank and step: P2P bytes, host and
                       # device time of the audit phase (inside the timed steps)
                       "audit_per_rank": [i.get("audit", {}) for i in inv_all],
                       "reassignments": [{"step": r["step"], "from_nodes": r["from_nodes"],
                                          "migration_ms": round(1000 * r["migration_time"], 2),
                                          "plan": r["plan"]} for r in engine.reassignment_history]},
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
    if _WATCHDOG is not None:
        _WATCHDOG.finish()
    if world > 1:
        dist.barrier()
        if _rec is not None:
            _rec.dump()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
