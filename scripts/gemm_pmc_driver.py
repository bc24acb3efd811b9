#!/usr/bin/env python3
"""Tiny GEMM driver for rocprofv3 --pmc passes: the qkv forward product (64k x 1024 x 3072) on the
native ping-pong kernel (tile order from TDL_GEMM_GROUPM) and on hipBLASLt, 5 launches each."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import gemm  # noqa: E402

M, K, N = int(os.environ.get("PMC_M", 65536)), int(os.environ.get("PMC_K", 1024)), int(os.environ.get("PMC_N", 3072))
a = ((torch.rand(M, K, device="cuda") * 2 - 1)).bfloat16()
b = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).bfloat16().t()
out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
gemm.KERNEL = os.environ.get("PMC_KERNEL", "pp")
for _ in range(5):
    gemm.matmul(a, b, out=out)
    torch.mm(a, b, out=out)
torch.cuda.synchronize()
print("done")
