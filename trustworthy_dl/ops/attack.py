"""In-place attack / fault injection (csrc/attack.hip) with a bit-compatible-in-spirit CPU path.

Modes (AttackMode): SCALE x*=a, NOISE x+=a*N(0,1), SIGN_FLIP x=-a*x, ZERO x=0,
REL_NOISE x*=(1+a*N(0,1)), SHIFT x+=a.  GPU noise is Philox4x32-10 keyed by (seed, offset),
so an injection is reproducible on any device, stream or graph replay.
"""
from __future__ import annotations

from enum import IntEnum

import torch

from . import _lib
from ._lib import ptr, stream_ptr


class AttackMode(IntEnum):
    SCALE = 0
    NOISE = 1
    SIGN_FLIP = 2
    ZERO = 3
    REL_NOISE = 4
    SHIFT = 5


def inject_(x: torch.Tensor, mode: AttackMode, intensity: float, seed: int = 0, offset: int = 0) -> torch.Tensor:
    if not x.is_contiguous():
        raise ValueError("attack injection needs a contiguous tensor")
    mode = AttackMode(mode)
    if x.is_cuda:
        code = _lib.DTYPE_CODE[x.dtype]
        if code not in (0, 1):
            raise TypeError(f"unsupported dtype {x.dtype}")
        _lib.call("tdl_attack_inject", ptr(x), code, x.numel(), int(mode), float(intensity),
                  seed & 0xFFFFFFFFFFFFFFFF, offset & 0xFFFFFFFFFFFFFFFF, stream_ptr(x.device))
        return x
    with torch.no_grad():
        if mode == AttackMode.SCALE:
            x.mul_(intensity)
        elif mode == AttackMode.SIGN_FLIP:
            x.mul_(-intensity)
        elif mode == AttackMode.ZERO:
            x.zero_()
        elif mode == AttackMode.SHIFT:
            x.add_(intensity)
        else:
            g = torch.Generator().manual_seed((seed * 1000003 + offset) & 0x7FFFFFFFFFFFFFFF)
            z = torch.randn(x.shape, generator=g, dtype=torch.float32).to(x.dtype)
            if mode == AttackMode.NOISE:
                x.add_(z * intensity)
            else:
                x.mul_(1 + intensity * z)
    return x
