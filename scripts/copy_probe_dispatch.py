"""Python stacks of the small device copies in one training step (TorchDispatchMode): which engine
code issues the ~100 tiny copy / fill kernels per step.  PROBE_MODULE=bench_cnn | bench."""
import collections
import importlib
import os
import sys
import traceback

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

bench = importlib.import_module(os.environ.get("PROBE_MODULE", "bench_cnn"))
from trustworthy_dl.parallel import pipeline  # noqa: E402

seen = collections.Counter()
OPS = ("copy_", "_to_copy", "fill_", "zero_", "clone", "lift_fresh", "_local_scalar_dense", "index_put_", "scalar_tensor")


class Probe(TorchDispatchMode):
    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__.split(".")[0]
        if name in OPS:
            shp = tuple(args[0].shape) if args and torch.is_tensor(args[0]) else None
            if shp is None or (len(shp) <= 1 and (not shp or shp[0] <= 64)):
                st = [f for f in traceback.extract_stack()[:-1] if "torch/" not in f.filename and "copy_probe" not in f.filename]
                key = " <- ".join(f"{os.path.relpath(f.filename)}:{f.lineno}" for f in st[-3:][::-1])
                seen[(name, str(shp), key)] += 1
        return func(*args, **(kwargs or {}))


orig = pipeline.PipelineEngine.train_step
state = {"n": 0}


def step(self, batch):
    state["n"] += 1
    if state["n"] != 5:
        return orig(self, batch)
    with Probe():
        out = orig(self, batch)
    return out


pipeline.PipelineEngine.train_step = step
sys.argv = [os.environ.get("PROBE_MODULE", "bench_cnn") + ".py", "--steps", "3", "--warmup", "3"]
bench.main()
for (n, shp, st), c in seen.most_common(40):
    print(c, n, shp, st, file=sys.stderr)
