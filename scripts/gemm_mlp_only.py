#!/usr/bin/env python3
"""PMC driver: the two fused MLP products on the native LDS-epilogue GEMM (variant 36) and the
library GEMMs of the same shapes, a few launches each (scripts/gpu_pmc_gemm.sh PROGS=gemm_mlp_only)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import _lib, gemm  # noqa: E402

_lib.lib()
gemm.VARIANT = 36
dev = torch.device("cuda:0")
M, C = 32768, 1024
r = lambda *s, sc=1.0: ((torch.rand(*s, device=dev) * 2 - 1) * sc).bfloat16()
h2, wfc_t, bfc = r(M, C), r(4 * C, C, sc=0.05), r(4 * C, sc=0.1)
dy, wp = r(M, C), r(4 * C, C, sc=0.05)
pre = torch.empty(M, 4 * C, dtype=torch.bfloat16, device=dev)
db = torch.zeros(4 * C, device=dev)
for _ in range(5):
    gemm.matmul(h2, wfc_t.t(), bias=bfc, epi="gelu", aux=pre)          # fc forward + bias + GELU
    gemm.matmul(dy, wp.t(), epi="dgelu", aux=pre, colsum=db)           # proj dgrad + dGELU + colsum
    torch.mm(h2, wfc_t.t())                                            # library, same shapes
    torch.mm(dy, wp.t())
torch.cuda.synchronize()
print("ok")
