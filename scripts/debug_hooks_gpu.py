import torch, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.models import get_model
from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
from trustworthy_dl.parallel.flat import AdamWConfig
m = get_model("gpt2-tiny", seq_len=128, seed=0, vocab_size=1024)
e = PipelineEngine(m, EngineConfig(num_nodes=2, micro_batches=2, seq_len=128, device="cuda:0", reassign=False,
                                   adamw=AdamWConfig(lr=1e-3), output_check="first"))
calls = {}
for n, st in e.stages.items():
    print(n, [type(r).__name__ for r in st._runners()], st._runner_layer_idx, getattr(st, "_layer_seg_runs", None))
    orig = st._grad_ready
    st._grad_ready = (lambda k, n=n, orig=orig: calls.setdefault(n, []).append(k) or orig(k))
    v = st.verifier
    og = v.grad_ready
    v.grad_ready = (lambda g, runs, n=n, og=og: calls.setdefault(f"v{n}", []).append((runs, v.verify_on, g.is_cuda)) or og(g, runs))
ids = torch.randint(0, 1024, (8, 129))
e.train_step({"input": ids[:, :-1], "target": ids[:, 1:]})
torch.cuda.synchronize()
print(calls)
