"""A few causal attention fwd+bwd launches at GPT-2-medium shape (for rocprofv3 PMC passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops.layers import attn_bwd, attn_fwd  # noqa: E402

B, H, T = int(os.environ.get("B", "32")), 16, 1024
qkv = torch.randn(B, T, 3 * H * 64, device="cuda").bfloat16()
for _ in range(3):
    o, lse, sc = attn_fwd(qkv, H, True)
    attn_bwd(qkv, o, lse, torch.randn_like(o), H, True, sc)
torch.cuda.synchronize()
print("done")
