"""The fused single-autograd-node GPT-2 block (ops/block.py) computes exactly what the
op-by-op module composition computes (CPU fp32: same primitives, hand-scheduled backward)."""
import copy

import torch

from trustworthy_dl.models.gpt2 import GPT2Block, GPT2Config


def _pair():
    torch.manual_seed(0)
    blk = GPT2Block(GPT2Config.from_size("tiny"))
    for p in blk.parameters():
        torch.nn.init.normal_(p, std=0.1)
    ref = copy.deepcopy(blk)
    ref.fused = False
    return blk, ref


def test_fused_block_forward_backward_match():
    blk, ref = _pair()
    x = torch.randn(2, 16, 128, requires_grad=True)
    xr = x.detach().clone().requires_grad_(True)
    y, yr = blk(x), ref(xr)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    assert torch.allclose(y, yr, atol=1e-5)
    assert torch.allclose(x.grad, xr.grad, atol=1e-5)
    for (n, p), (_, q) in zip(blk.named_parameters(), ref.named_parameters()):
        assert torch.allclose(p.grad, q.grad, atol=1e-5, rtol=1e-4), n


def test_fused_block_main_grad_accumulates():
    blk, ref = _pair()
    for p in blk.parameters():
        p.main_grad = torch.zeros_like(p)
    x = torch.randn(2, 16, 128)
    for _ in range(2):  # two micro-batches accumulate
        blk(x.clone().requires_grad_(True)).sum().backward()
        ref(x.clone().requires_grad_(True)).sum().backward()
    for (n, p), (_, q) in zip(blk.named_parameters(), ref.named_parameters()):
        assert p.grad is None
        assert torch.allclose(p.main_grad, q.grad, atol=1e-4, rtol=1e-4), n
