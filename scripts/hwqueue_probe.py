"""Measure false dependencies between HIP streams that share a hardware queue.

For every ordered pair (X, Y) of streams — the null stream the pipeline computes on plus
``--streams`` streams from torch's pool (the pool RCCL's communicator streams come from) — launch a
bounded spin-wait on X, then the kernel that releases it on Y.  ``blocked`` means Y's kernel ran
only after X's wait timed out: a kernel on Y queued behind a spinning kernel on X, which is what a
receive posted ahead of compute does to the compute stream when they share a queue.

Run with different GPU_MAX_HW_QUEUES (read by the HIP runtime at start-up):

    GPU_MAX_HW_QUEUES=4  python scripts/hwqueue_probe.py --out gpurun_out/hwq4.json
    GPU_MAX_HW_QUEUES=16 python scripts/hwqueue_probe.py --out gpurun_out/hwq16.json

Build: hipcc --offload-arch=gfx950 -O2 -shared -fPIC scripts/hwqueue_probe.hip -o scripts/libhwqueue_probe.so
"""
import argparse
import ctypes
import json
import os
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=12)
    ap.add_argument("--timeout-ms", type=float, default=30.0)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    lib = ctypes.CDLL(os.path.join(HERE, "libhwqueue_probe.so"))
    lib.probe_pair.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    lib.probe_pair.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    ticks = int(args.timeout_ms * 1e-3 * 100e6)  # wall_clock64 runs at 100 MHz on CDNA3/4
    streams = [("null", torch.cuda.default_stream(dev))]
    streams += [(f"pool{i}", torch.cuda.Stream(dev)) for i in range(args.streams)]
    n = len(streams)
    flags = torch.zeros(n * n, dtype=torch.int32, device=dev)
    outs = torch.zeros(n * n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    blocked = []
    t0 = time.time()
    for a, (na, sa) in enumerate(streams):
        for b, (nb, sb) in enumerate(streams):
            if a == b:
                continue
            k = a * n + b
            f = flags.data_ptr() + 4 * k
            rc = lib.probe_pair(ctypes.c_void_p(f), ctypes.c_void_p(f), ctypes.c_void_p(outs.data_ptr() + 4 * k),
                                ctypes.c_uint64(ticks), ctypes.c_void_p(sa.cuda_stream), ctypes.c_void_p(sb.cuda_stream))
            assert rc == 0, f"launch failed rc={rc}"
            torch.cuda.synchronize()
    res = outs.view(n, n).cpu()
    for a in range(n):
        for b in range(n):
            if a != b and int(res[a, b]) == 2:
                blocked.append([streams[a][0], streams[b][0]])
    # streams whose kernels serialise behind each other in BOTH orders share a queue
    groups = {}
    for a in range(n):
        key = tuple(int(res[a, b]) == 2 or a == b for b in range(n))
        groups.setdefault(key, []).append(streams[a][0])
    summary = {
        "GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES", "default"),
        "streams": n, "pairs": n * (n - 1), "blocked_pairs": len(blocked),
        "null_blocked_behind": [x for x, y in blocked if y == "null"],
        "blocked_behind_null": [y for x, y in blocked if x == "null"],
        "queue_groups": sorted(groups.values(), key=len, reverse=True),
        "unset": int((res == 0).sum()) - n,
        "seconds": round(time.time() - t0, 2),
    }
    print(json.dumps(summary))
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as fh:
            json.dump({**summary, "blocked": blocked}, fh, indent=1)


if __name__ == "__main__":
    main()
