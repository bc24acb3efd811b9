"""Which Python call sites launch the small torch (at::native) kernels of a training step?  Runs a
bench's main (PROBE_MODULE=bench | bench_cnn) and, during ONE step after warm-up, wraps the torch
entry points that launch copy / fill / elementwise kernels (Tensor.to / copy_ / zero_ / fill_ /
add_ / float / contiguous, torch.zeros / zeros_like / cat) to count calls and bytes per call site.
Autograd's own C++ gradient accumulation is not seen (no Python frame).
Usage: PROBE_MODULE=bench_cnn python scripts/op_probe.py --model resnet50 --steps 3 --warmup 2"""
import collections
import importlib
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from trustworthy_dl.parallel import pipeline  # noqa: E402

bench = importlib.import_module(os.environ.get("PROBE_MODULE", "bench"))
TARGET = int(os.environ.get("PROBE_STEP", "4"))
stats = collections.defaultdict(lambda: [0, 0])
active = [False]


def site():
    fr = [f for f in traceback.extract_stack()[:-2] if "op_probe" not in f.filename]
    own = [f for f in fr if "/torch/" not in f.filename]
    f = own[-1] if own else fr[-1]
    return f"{os.path.relpath(f.filename)}:{f.lineno} {f.line}"


def wrap(owner, name):
    fn = getattr(owner, name)

    def w(*a, **k):
        out = fn(*a, **k)
        if active[0]:
            t = out if isinstance(out, torch.Tensor) else (a[0] if a and isinstance(a[0], torch.Tensor) else None)
            if t is not None and t.is_cuda:
                s = stats[(name, site())]
                s[0] += 1
                s[1] += t.numel() * t.element_size()
        return out
    setattr(owner, name, w)


for n in ("to", "copy_", "zero_", "fill_", "add_", "float", "contiguous", "clone", "__setitem__"):
    wrap(torch.Tensor, n)
for n in ("zeros", "zeros_like", "cat"):
    wrap(torch, n)

orig = pipeline.PipelineEngine.train_step


def step(self, batch):
    step.n += 1
    active[0] = step.n == TARGET
    try:
        if not active[0]:
            return orig(self, batch)
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU], record_shapes=True) as p:
            out = orig(self, batch)
        step.prof = p
        return out
    finally:
        active[0] = False


step.n = 0
step.prof = None
pipeline.PipelineEngine.train_step = step
bench.main()
for (name, where), (n, b) in sorted(stats.items(), key=lambda kv: -kv[1][1])[:50]:
    print(f"{b / 1e6:10.2f} MB  n={n:4d}  {name:10s} {where}", file=sys.stderr)

# C++-originated launches (no Python frame): the autograd function each op ran under
if step.prof is not None:
    agg = collections.Counter()
    for e in step.prof.events():
        if e.name not in ("aten::to", "aten::add_", "aten::fill_", "aten::zero_", "aten::copy_", "aten::zeros"):
            continue
        par, chain = e.cpu_parent, []
        while par is not None:
            chain.append(par.name)
            par = par.cpu_parent
        top = next((c for c in chain if c.startswith("autograd::engine::evaluate_function")), chain[-1] if chain else "-")
        agg[(e.name, top[:90], str(e.input_shapes)[:80], str(getattr(e, "input_types", ""))[:0])] += 1
    for (name, top, shp, _), n in agg.most_common(40):
        print(f"n={n:4d} {name:12s} under {top}  shapes={shp}", file=sys.stderr)
