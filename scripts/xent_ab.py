#!/usr/bin/env python3
"""Fused LM-head cross-entropy pass (tdl_xent_fused: loss, lse, dlogits in place) at the bench shape
[65536, 50304] (V = 50257): us per call and effective TB/s of one read + one write of the logits.
Run once per library build (TDL_NATIVE_LIB) for an A/B of two builds; prints one JSON line."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import _lib  # noqa: E402
from trustworthy_dl.ops._lib import ptr, stream_ptr  # noqa: E402

M, V, ld = 65536, 50257, 50304
torch.manual_seed(0)
base = (torch.randn(M, ld, device="cuda") * 2).bfloat16()
labels = torch.randint(0, V, (M,), device="cuda")
labels[::7] = -100
loss = torch.empty(M, device="cuda")
lse = torch.empty(M, device="cuda")
scale = torch.tensor([1.0 / M], device="cuda")
x = base.clone()


def run():
    _lib.call("tdl_xent_fused", ptr(x), ptr(labels), ptr(loss), ptr(lse), ptr(scale), M, V, ld, stream_ptr(x.device))


run()
torch.cuda.synchronize()
rows = slice(0, 512)
lf = base[rows, :V].float()
ref_lse = torch.logsumexp(lf, -1)
err_lse = float((lse[rows] - ref_lse).abs().max())
p = torch.softmax(lf, -1)
lab = labels[rows]
ok = lab >= 0
p[ok.nonzero().squeeze(1), lab[ok]] -= 1.0
p[~ok] = 0
ref_dl = p / M
err_dl = float((x[rows, :V].float() - ref_dl).abs().max() / ref_dl.abs().max())
ts = []
for _ in range(5):
    x.copy_(base)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    run()
    e.record()
    e.synchronize()
    ts.append(s.elapsed_time(e) * 1e3)
us = statistics.median(ts)
print(json.dumps({"lib": os.environ.get("TDL_NATIVE_LIB", "default"), "us": round(us, 1),
                  "TB_s_rw": round(2 * M * ld * 2 / us / 1e6, 2), "err_lse": err_lse, "err_dlogits": err_dl}), flush=True)
