import os, sys, collections
sys.path.insert(0, os.getcwd())
import torch
from torch.profiler import profile, ProfilerActivity
import importlib
bench = importlib.import_module(os.environ.get("PROBE_MODULE", "bench"))   # or bench_cnn
from trustworthy_dl.parallel import pipeline
orig = pipeline.PipelineEngine.train_step
state = {"n": 0, "prof": None}
def step(self, batch):
    state["n"] += 1
    if state["n"] != 5:
        return orig(self, batch)
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True, record_shapes=True) as p:
        out = orig(self, batch)
        torch.cuda.synchronize()
    state["prof"] = p
    return out
pipeline.PipelineEngine.train_step = step
sys.argv = [os.environ.get("PROBE_MODULE", "bench") + ".py", "--steps", "3", "--warmup", "3"]
bench.main()
p = state["prof"]
ka = p.key_averages(group_by_stack_n=8)
rows = [e for e in ka if e.key in ("aten::copy_", "aten::to", "aten::_to_copy", "aten::clone", "aten::contiguous", "aten::index_put_", "aten::index", "aten::cat", "aten::stack", "aten::fill_", "aten::zero_", "aten::add", "aten::add_", "aten::zeros", "aten::zeros_like")]
rows.sort(key=lambda e: -e.count)
for e in rows[:25]:
    st = [s for s in (e.stack or []) if "torch/" not in s][:4]
    print(e.count, e.key, round(e.device_time_total if hasattr(e, "device_time_total") else e.cuda_time_total, 1), " | ".join(st), file=sys.stderr)

print("--- by input shape", file=sys.stderr)
ks = p.key_averages(group_by_input_shape=True)
rows = [e for e in ks if e.key in ("aten::copy_", "aten::_to_copy", "aten::add_", "aten::clone", "aten::contiguous")]
rows.sort(key=lambda e: -(e.device_time_total if hasattr(e, "device_time_total") else e.cuda_time_total))
for e in rows[:25]:
    print(e.count, e.key, round(e.device_time_total if hasattr(e, "device_time_total") else e.cuda_time_total, 1), str(e.input_shapes)[:160], file=sys.stderr)

print("--- small copies with Python stacks", file=sys.stderr)
seen = collections.Counter()
for e in p.events():
    if e.name in ("aten::copy_", "aten::_to_copy", "aten::fill_", "aten::zero_") and e.input_shapes and e.input_shapes[0] in ([1], [], [2]):
        st = [s for s in (e.stack or []) if "torch/" not in s and "<built-in" not in s][:5]
        seen[(e.name, str(e.input_shapes[0]), " | ".join(st))] += 1
for (n, sh, st), c in seen.most_common(30):
    print(c, n, sh, st, file=sys.stderr)
