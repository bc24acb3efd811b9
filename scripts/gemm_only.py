#!/usr/bin/env python3
"""Driver for rocprofv3 counter passes: native GEMM (shipped schedule) vs hipBLASLt (torch.mm) on the
GPT-2-medium NT shapes proj fwd (K=4096) and fc fwd (K=1024), 5 calls each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import gemm  # noqa: E402

dev = torch.device("cuda:0")
M = 32768
r = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).bfloat16()
xp, wp = r(M, 4096), r(1024, 4096)
xf, wf = r(M, 1024), r(4096, 1024)
variant = int(os.environ.get("GEMM_VARIANT", "0"))
for _ in range(5):
    gemm.VARIANT = variant
    gemm.matmul(xp, wp.t())
    gemm.matmul(xf, wf.t())
    torch.mm(xp, wp.t())
    torch.mm(xf, wf.t())
torch.cuda.synchronize()
print("ok")
