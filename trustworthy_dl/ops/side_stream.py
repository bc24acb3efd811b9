"""Side HIP stream for weight-gradient work that runs beside the input-gradient chain."""
from __future__ import annotations

import os

import torch


class WgradSide:
    """Weight gradients on a second HIP stream.

    A layer's input gradient and weight gradient both need only dY: the input gradient stays on
    the compute stream (the backward's critical path) and the weight gradient runs beside it
    (convolutions: ops/conv.py, ``TDL_CONV_WGRAD_SIDE=0`` turns it off).  ResNet-50's 14 x 14 / 7 x 7 layers launch 196 / 100 data-gradient workgroups on 256 CUs, so the
    weight gradient fills CUs that would idle: +5.3 % images/s (profiles/r4_conv_wgrad_side_ab.txt).
    The GPT-2 block's weight-gradient GEMMs were tried the same way and measured +0.04 % (their
    input-gradient GEMMs already fill the chip: profiles/r4_gemm_wgrad_side_ab.txt), so they stay
    inline.  Ordering: every consumer of a weight gradient
    waits for this stream — the backward pass itself at its end (an autograd final callback makes
    the compute stream wait) and the verifier's side stream before it takes per-layer gradient
    statistics mid-backward and the tied-gradient all-reduce (``wait_wgrad``).  The caller lists
    the tensors the work reads (``keep``) so the caching allocator holds them until it is done."""
    streams = {}
    pending = {}

    @staticmethod
    def on(var: str, default: str) -> bool:
        return os.environ.get(var, default) != "0"

    @classmethod
    def run(cls, dev: torch.device, fn, keep):
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        side = cls.streams.get(idx)
        if side is None:
            side = cls.streams[idx] = torch.cuda.Stream(device=dev)
        cur = torch.cuda.current_stream(dev)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            fn()
        for t in keep:
            if t is not None:
                t.record_stream(side)
        if not cls.pending.get(idx):
            cls.pending[idx] = True

            def _join(idx=idx, cur=cur, side=side):
                cur.wait_stream(side)
                cls.pending[idx] = False
            torch.autograd.Variable._execution_engine.queue_callback(_join)

    @classmethod
    def join_all(cls):
        """Make each device's current stream wait for its side stream and clear the pending flags:
        called by the engine at every step start, so a backward that raised after a side-stream
        launch (its final callback never ran) cannot leave the next step's consumers unordered
        (ADVICE r4)."""
        for idx, side in cls.streams.items():
            if cls.pending.get(idx):
                torch.cuda.current_stream(torch.device("cuda", idx)).wait_stream(side)
                cls.pending[idx] = False

    @classmethod
    def count(cls) -> int:
        return len(cls.streams)

    @classmethod
    def wait(cls, stream: torch.cuda.Stream, dev: torch.device):
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        if cls.pending.get(idx):
            stream.wait_stream(cls.streams[idx])


def wait_wgrad(stream, dev: torch.device):
    """Make ``stream`` wait for the weight gradients issued so far on the side stream."""
    WgradSide.wait(stream, dev)
