"""Where does the training step block the host on the GPU?  Runs bench.py's main with torch's CUDA
sync debug mode on and prints every distinct Python stack that triggered a synchronising call
(with its count).  Usage: python scripts/sync_probe.py --steps 3 --warmup 2 (bench.py arguments);
PROBE_MODULE=bench_cnn probes the conv-net bench instead."""
import collections
import os
import sys
import traceback
import warnings

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import importlib  # noqa: E402

bench = importlib.import_module(os.environ.get("PROBE_MODULE", "bench"))

seen = collections.Counter()


def hook(message, category, filename, lineno, file=None, line=None):
    if "synchroniz" not in str(message):
        return
    st = [f for f in traceback.extract_stack()[:-1] if "warnings" not in f.filename]
    key = "".join(f"    {os.path.relpath(f.filename)}:{f.lineno} {f.name}: {f.line}\n" for f in st[-7:])
    seen[(str(message)[:80], key)] += 1


warnings.simplefilter("always")
warnings.showwarning = hook
torch.cuda.set_sync_debug_mode("warn")
try:
    bench.main()
finally:
    torch.cuda.set_sync_debug_mode(0)
    for (msg, st), n in seen.most_common(40):
        print(f"== {n}x {msg}\n{st}", file=sys.stderr)
