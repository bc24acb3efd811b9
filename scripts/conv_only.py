"""A few native conv fwd/dgrad/wgrad launches at a ResNet-50 3x3 shape (for rocprofv3 PMC passes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops.conv import conv2d  # noqa: E402

x = torch.randn(32, 128, 28, 28, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last)
x.requires_grad_(True)
w = (torch.randn(128, 128, 3, 3, device="cuda") * 0.05).bfloat16().requires_grad_(True)
for _ in range(3):
    y = conv2d(x, w, 1, 1)
    y.backward(torch.ones_like(y))
torch.cuda.synchronize()
print("done")
