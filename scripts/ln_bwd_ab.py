#!/usr/bin/env python3
"""LayerNorm backward (tdl_layernorm_bwd_res, the pre-LN block's fused residual / bias-sum form) at
the bench shape [65536, 1024]: us per call and effective TB/s of the 512 MB it must move.  Run once
per library build (TDL_NATIVE_LIB) for an A/B of two builds; prints one JSON line."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import block  # noqa: E402

M, N = 65536, 1024
torch.manual_seed(0)
x = torch.randn(M, N, device="cuda").bfloat16()
dy = torch.randn(M, N, device="cuda").bfloat16()
dres = torch.randn(M, N, device="cuda").bfloat16()
w = (1 + 0.1 * torch.randn(N, device="cuda")).bfloat16()
mean = x.float().mean(-1)
rstd = torch.rsqrt(x.float().var(-1, unbiased=False) + 1e-5)
acc = [torch.zeros(N, device="cuda") for _ in range(4)]
dx = block._ln_bwd(dy, x, w, mean, rstd, acc[0], acc[1], dres=dres, sres_acc=acc[2], sdx_acc=acc[3])
# reference
xh = (x.float() - mean[:, None]) * rstd[:, None]
gw = dy.float() * w.float()
ref = rstd[:, None] * (gw - gw.mean(-1, keepdim=True) - xh * (gw * xh).mean(-1, keepdim=True)) + dres.float()
err = float((dx.float() - ref).abs().max() / ref.abs().max())
ts = []
for _ in range(5):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        block._ln_bwd(dy, x, w, mean, rstd, acc[0], acc[1], dres=dres, sres_acc=acc[2], sdx_acc=acc[3])
    e.record()
    e.synchronize()
    ts.append(s.elapsed_time(e) * 1e3 / 20)
us = statistics.median(ts)
print(json.dumps({"lib": os.environ.get("TDL_NATIVE_LIB", "default"), "us": round(us, 1),
                  "TB_s": round(4 * M * N * 2 / us / 1e6, 2), "relerr": err}), flush=True)
