#!/usr/bin/env python3
"""Microbenchmark: native implicit-GEMM MFMA conv (csrc/conv.hip) vs MIOpen (torch conv, channels_last
bf16) on ResNet-50 / VGG layer shapes at batch 32 (224x224 ImageNet shape).  Prints one JSON line
per shape: forward / dgrad / wgrad TFLOP/s for both paths.  Interleaved rounds in one process."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from trustworthy_dl.ops import _lib  # noqa: E402
from trustworthy_dl.ops._lib import ptr, stream_ptr  # noqa: E402
from trustworthy_dl.ops.conv import _num_cu  # noqa: E402

# name, N, C, H, Cout, R, stride, pad
SHAPES = [
    ("r50.s1.3x3", 32, 64, 56, 64, 3, 1, 1),
    ("r50.s1.1x1a", 32, 64, 56, 256, 1, 1, 0),
    ("r50.s1.1x1b", 32, 256, 56, 64, 1, 1, 0),
    ("r50.s2.3x3", 32, 128, 28, 128, 3, 1, 1),
    ("r50.s3.3x3", 32, 256, 14, 256, 3, 1, 1),
    ("r50.s3.1x1", 32, 1024, 14, 256, 1, 1, 0),
    ("r50.s4.3x3", 32, 512, 7, 512, 3, 1, 1),
    ("r50.s4.1x1", 32, 512, 7, 2048, 1, 1, 0),
    ("r50.stem", 32, 8, 224, 64, 7, 2, 3),
    ("vgg.c3", 32, 256, 56, 256, 3, 1, 1),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    dev = torch.device("cuda:0")
    ncu = _num_cu(dev)
    for name, N, C, H, Co, R, st, pad in SHAPES:
        W = H
        P = (H + 2 * pad - R) // st + 1
        Q = P
        x = torch.randn(N, C, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(Co, C, R, R, device=dev) * 0.05).to(torch.bfloat16)
        wk = w.permute(0, 2, 3, 1).contiguous()
        wd = w.permute(1, 2, 3, 0).contiguous()
        wcl = w.contiguous(memory_format=torch.channels_last)
        y = torch.empty(N, Co, P, Q, device=dev, dtype=torch.bfloat16, memory_format=torch.channels_last)
        dy = torch.randn_like(y)
        dx = torch.empty_like(x)
        dw = torch.zeros(Co, C, R, R, device=dev, dtype=torch.float32)
        stats = torch.empty(2 * Co, device=dev)
        sws = torch.empty(int(_lib.lib().tdl_conv_stats_ws_floats(N * P * Q, Co)), device=dev)
        wws = torch.empty(Co * R * R * C, device=dev)
        flops = 2.0 * N * P * Q * Co * C * R * R
        s = stream_ptr(dev)
        fwd = lambda: _lib.call("tdl_conv_nt", ptr(x), ptr(wk), ptr(y), ptr(stats), ptr(sws), N, H, W, C, P, Q, Co, R, R,
                                st, pad, 0, s)
        fwd0 = lambda: _lib.call("tdl_conv_nt", ptr(x), ptr(wk), ptr(y), None, None, N, H, W, C, P, Q, Co, R, R, st, pad,
                                 0, s)
        dgr = lambda: _lib.call("tdl_conv_nt", ptr(dy), ptr(wd), ptr(dx), None, None, N, P, Q, Co, H, W, C, R, R, st,
                                pad, 1, s)
        wgr = lambda: _lib.call("tdl_conv_wgrad", ptr(dy), ptr(x), ptr(dw), ptr(wws), N, H, W, C, P, Q, Co, R, R, st,
                                pad, ncu, s)
        t_fwd, t_fwd0, t_dgr, t_wgr = timeit(fwd), timeit(fwd0), timeit(dgr), timeit(wgr)
        # MIOpen through torch (channels_last bf16)
        m_fwd = lambda: F.conv2d(x, wcl, None, st, pad)
        m_dgr = lambda: torch.ops.aten.convolution_backward(dy, x, wcl, None, (st, st), (pad, pad), (1, 1), False,
                                                           (0, 0), 1, (True, False, False))
        m_wgr = lambda: torch.ops.aten.convolution_backward(dy, x, wcl, None, (st, st), (pad, pad), (1, 1), False,
                                                           (0, 0), 1, (False, True, False))
        try:
            mt = (timeit(m_fwd), timeit(m_dgr), timeit(m_wgr))
        except Exception as e:  # noqa: BLE001
            mt = (float("nan"),) * 3
            print(f"miopen failed for {name}: {e}", file=sys.stderr)
        tf = lambda t: round(flops / t / 1e12, 1)
        print(json.dumps({"shape": name, "gflop": round(flops / 1e9, 2),
                          "native_tflops": {"fwd+stats": tf(t_fwd), "fwd": tf(t_fwd0), "dgrad": tf(t_dgr), "wgrad": tf(t_wgr)},
                          "miopen_tflops": {"fwd": tf(mt[0]), "dgrad": tf(mt[1]), "wgrad": tf(mt[2])},
                          "native_us": [round(t_fwd * 1e6, 1), round(t_dgr * 1e6, 1), round(t_wgr * 1e6, 1)]}),
              flush=True)


if __name__ == "__main__":
    main()
