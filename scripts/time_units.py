#!/usr/bin/env python3
"""Per-pipeline-unit fwd+bwd time of GPT-2-medium on one GPU (calibrates GPT2LMHeadModel.layer_costs).

Builds real pipeline Stages (flat fp32 master + main_grad accumulation, bf16 compute) holding one
unit each — embedding, attention half, MLP half, a fused (attn, mlp) pair, a whole block, the
ln_f + LM head + cross-entropy — and times forward + backward of one micro-batch.  Prints one JSON
line per unit with ms and the ratio to the whole block."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.models import get_model  # noqa: E402
from trustworthy_dl.parallel.stage import Stage  # noqa: E402


def time_stage(st, x, labels, iters=10):
    def step():
        xi = x.detach().requires_grad_(x.is_floating_point())
        y, _ = st.forward(xi, labels)
        if st.computes_loss:
            y.backward()
        else:
            y.backward(torch.ones_like(y))
    for _ in range(3):
        step()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        step()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda:0")
    mbs = int(os.environ.get("MBS", "16"))
    T = 1024
    model = get_model("gpt2-medium", seq_len=T, seed=0)
    n = model.config.n_embd
    ids = torch.randint(0, 50257, (mbs, T), device=dev)
    h = (torch.randn(mbs, T, n, device=dev) * 0.5).bfloat16()
    res = {}
    model.set_pipeline_granularity("block")
    L = len(model.pipeline_layers())
    units = {"block": ((1, 2), h, None), "head": ((L - 1, L), h, ids), "embed": ((0, 1), ids, None)}
    for name, (rng, x, lab) in units.items():
        st = Stage(model, rng, 0, 1, dev, torch.bfloat16)
        res[name] = time_stage(st, x, lab)
        del st
    model.set_pipeline_granularity("half")
    for name, rng in {"attn_half": (1, 2), "mlp_half": (2, 3), "pair": (1, 3)}.items():
        st = Stage(model, rng, 0, 1, dev, torch.bfloat16)
        res[name] = time_stage(st, h, None)
        del st
    for k, v in res.items():
        print(json.dumps({"unit": k, "mbs": mbs, "ms": round(v, 3), "vs_block": round(v / res["block"], 3)}),
              flush=True)
    c_blk = model.layer_costs(T)
    print(json.dumps({"model_costs_vs_block": {"attn": round(c_blk[1] / (c_blk[1] + c_blk[2]), 3),
                                               "mlp": round(c_blk[2] / (c_blk[1] + c_blk[2]), 3),
                                               "head": round(c_blk[-1] / (c_blk[1] + c_blk[2]), 3)}}))


if __name__ == "__main__":
    main()
