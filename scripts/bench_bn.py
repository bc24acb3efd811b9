"""Microbenchmark of the native BatchNorm(+ReLU) passes on ResNet-50's stored-output BN shapes
(NHWC bf16, batch 64): forward apply, backward reduce + fold + dx (tdl_bn_act_bwd).  Prints one JSON
line per shape with us/call and the effective HBM bandwidth (bytes each pass must move).
BN_LABEL tags the output lines (A/B of builds)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import _lib  # noqa: E402
from trustworthy_dl.ops._lib import ptr, stream_ptr  # noqa: E402

SHAPES = [(64 * 112 * 112, 64, False), (64 * 56 * 56, 256, True), (64 * 28 * 28, 512, True),
          (64 * 14 * 14, 1024, True), (64 * 7 * 7, 2048, True)]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000.0 / iters


def main():
    dev = torch.device("cuda")
    L = _lib.lib()
    for M, C, res in SHAPES:
        x = torch.randn(M, C, device=dev).bfloat16()
        r = torch.randn(M, C, device=dev).bfloat16() if res else None
        dout = torch.randn(M, C, device=dev).bfloat16()
        xf = x.float()
        stats = torch.cat([xf.sum(0), (xf * xf).sum(0)]).contiguous()
        gamma = (1 + 0.1 * torch.randn(C, device=dev)).bfloat16()
        beta = (0.1 * torch.randn(C, device=dev)).bfloat16()
        out = torch.empty_like(x)
        mean = torch.empty(C, device=dev)
        rstd = torch.empty(C, device=dev)
        ws = torch.zeros(int(L.tdl_bn_bwd_ws_floats(C)), device=dev)
        part = torch.empty(int(L.tdl_bn_bwd_part_floats(C)), device=dev)
        dx, dres = torch.empty_like(x), (torch.empty_like(x) if res else None)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        s = stream_ptr(dev)

        def fwd():
            _lib.call("tdl_bn_act_fwd", ptr(x), ptr(stats), None, None, ptr(gamma), ptr(beta), ptr(r), ptr(out),
                      ptr(mean), ptr(rstd), None, None, ptr(ws), M, C, 1e-5, 0.1, 1, s)

        def bwd():
            ws.zero_()
            _lib.call("tdl_bn_act_bwd", ptr(dout), ptr(out), ptr(x), ptr(mean), ptr(rstd), ptr(gamma), ptr(ws), ptr(part),
                      ptr(dx), ptr(dres), ptr(dg), ptr(db), M, C, 1, s)

        def zero():
            ws.zero_()

        fwd()
        t_f = timeit(fwd)
        t_b = timeit(bwd) - timeit(zero)
        el = M * C * 2
        # fwd: x (+res) in, out; bwd: reduce reads dout, out, x; dx pass reads dout, out, x, writes dx (+dres)
        by_f = el * (3 if res else 2)
        by_b = el * (3 + 4 + (1 if res else 0))
        print(json.dumps({"M": M, "C": C, "res": res, "build": os.environ.get("BN_LABEL", ""),
                          "fwd_us": round(t_f, 1), "fwd_TBps": round(by_f / t_f / 1e6, 2),
                          "bwd_us": round(t_b, 1), "bwd_TBps": round(by_b / t_b / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
