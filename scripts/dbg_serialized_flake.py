"""Debug: repeat tests/test_engine_gpu.py::test_serialized_streams_match_overlapped in one process and
report which digest slots differ when the overlapped and serialized runs disagree."""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import test_engine_gpu as T  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
for r in range(n):
    _, l0, d0, w0 = T._run(serialize_streams=False, output_check="first")
    _, l1, d1, w1 = T._run(serialize_streams=True, output_check="first")
    diff = (d0 - d1).abs()
    bad = (diff > 1e-6 + 1e-5 * d1.abs()).nonzero().tolist()
    print(r, "loss", l0, l1, "maxdiff", float(diff.max()), "wdiff", float((w0 - w1).abs().max()),
          "bad", [(i, j, float(d0[i, j]), float(d1[i, j])) for i, j in bad[:8]], flush=True)
