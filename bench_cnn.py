#!/usr/bin/env python3
"""Conv-net pipeline benchmark (BASELINE.json config 4 family): ResNet / VGG model-parallel training with
gradient verification + output detection on, bf16 on the native NHWC implicit-GEMM conv kernels,
synthetic ImageNet-shape (or CIFAR-shape) images, random-init weights.  Reports images/s.

    python bench_cnn.py --model resnet50 --image-size 224 --batch-per-gpu 64
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench_cnn.py --gpus N

Same timing protocol as bench.py: W untimed steps, barrier + device sync, K timed optimizer steps,
barrier + device sync, MAX over ranks; weak scaling (global batch = batch-per-gpu x N).
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--batch-per-gpu", type=int, default=64)
    ap.add_argument("--micro-batches", type=int, default=0, help="0 = 1 per stage x 4 (pipelined), 1 at N=1")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--lr", type=float, default=None,
                    help="AdamW lr (default 1e-3 for ResNets, 1e-4 for VGG: the 25088->4096->4096 classifier "
                         "diverges at 1e-3 in fp32 on the CPU too, profiles/r2_vgg16_lr_cpu_fp32.json)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
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
    gb = args.batch_per_gpu * N
    M = args.micro_batches or (1 if N == 1 else 4 * N)
    while gb % M:
        M -= 1
    name = args.model
    model = get_model(name, image_size=args.image_size, seed=1234)
    ncls = model.pipeline_layers()[-1].num_classes
    verify = not args.no_verify
    lr = args.lr if args.lr is not None else (1e-4 if name.startswith("vgg") else 1e-3)
    cfg = EngineConfig(num_nodes=N, micro_batches=M, adamw=AdamWConfig(lr=lr, weight_decay=1e-4, max_grad_norm=1.0),
                       attack_detection=verify, gradient_verification=verify, quarantine=verify, reassign=False)
    engine = PipelineEngine(model, cfg)
    del model
    g = torch.Generator().manual_seed(0)
    batches = []
    for _ in range(2):
        x = torch.randn(gb, 3, args.image_size, args.image_size, generator=g)
        y = torch.randint(0, ncls, (gb,), generator=g)
        batches.append({"input": x.pin_memory() if use_cuda else x, "target": y.pin_memory() if use_cuda else y})

    def sync():
        if world > 1:
            dist.barrier()
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
    for i in range(args.warmup):
        engine.train_step(next(feed))
    engine.flush()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        engine.train_step(next(feed))
    sync()
    elapsed = time.perf_counter() - t0
    engine.flush()
    el = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}" if use_cuda else "cpu")
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el)
    if rank == 0:
        print(json.dumps({
            "metric": f"images/sec {args.model} MP={N} with grad-verify on", "value": round(gb * args.steps / elapsed, 1),
            "unit": "images/s", "n_gpus": N, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1000 * elapsed / args.steps, 3), "higher_is_better": True, "scaling": "weak",
            "dtype": "bf16", "data": "synthetic images, random-init weights",
            "config": {"model": name, "global_batch": gb, "image_size": args.image_size, "micro_batches": M,
                       "parallelism": f"pp{N}", "grad_verify": verify, "plan": engine.plan.describe(), "lr": lr,
                       "last_loss": engine.last_loss}}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
