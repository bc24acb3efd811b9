#!/usr/bin/env python3
"""Tiny weight-gradient driver for rocprofv3 --pmc passes: the qkv weight gradient of GPT-2-medium
at 64k tokens (fp32 main_grad += x^T dy, [1024 x 65536] @ [65536 x 3072]) on the persistent kernel
(gemm_p4, split-K slabs + reduce), 5 launches.  PMC_KERNEL=p4|pd picks the kernel, PMC_NT=1 feeds it
pre-transposed (k-contiguous) operands instead of the stored [tokens][features] ones."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import gemm  # noqa: E402

T, C, N = int(os.environ.get("PMC_T", 65536)), int(os.environ.get("PMC_C", 1024)), int(os.environ.get("PMC_N", 3072))
x = ((torch.rand(T, C, device="cuda") * 2 - 1)).bfloat16()
dy = ((torch.rand(T, N, device="cuda") * 2 - 1) * 0.05).bfloat16()
acc = torch.zeros(C, N, dtype=torch.float32, device="cuda")
KN = os.environ.get("PMC_KERNEL", "p4")
if KN == "grouped":    # the qkv + o pair from one grouped launch (gemm.matmul_f32_acc_grouped)
    o = ((torch.rand(T, C, device="cuda") * 2 - 1)).bfloat16()
    dy1 = ((torch.rand(T, C, device="cuda") * 2 - 1) * 0.05).bfloat16()
    acc_o = torch.zeros(C, C, dtype=torch.float32, device="cuda")
    N = N + C

    def _grouped(acc, a_op, b_op, kernel=None):
        assert gemm.matmul_f32_acc_grouped(acc, a_op, b_op, acc_o, o.t(), dy1)
    gemm.matmul_f32_acc = _grouped
if os.environ.get("PMC_NT", "0") == "1":
    a_op, b_op = x.t().contiguous(), dy.t().contiguous().t()
else:
    a_op, b_op = x.t(), dy
for _ in range(5):
    gemm.matmul_f32_acc(acc, a_op, b_op, kernel=KN)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10):
    gemm.matmul_f32_acc(acc, a_op, b_op, kernel=KN)
e.record()
e.synchronize()
ms = s.elapsed_time(e) / 10
print(f"done {ms * 1e3:.1f} us/call {2.0 * T * C * N / ms / 1e9:.1f} TF/s", flush=True)
