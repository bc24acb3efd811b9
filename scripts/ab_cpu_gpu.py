import torch, sys
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from trustworthy_dl.models import get_model
from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
from trustworthy_dl.parallel.flat import AdamWConfig
from trustworthy_dl.utils.metrics import MetricsCollector
def run(verify):
    m = get_model("gpt2-tiny", seq_len=128, seed=1234)
    cfg = EngineConfig(num_nodes=1, micro_batches=2, seq_len=128, device=sys.argv[1] if len(sys.argv) > 1 else "cpu",
                       adamw=AdamWConfig(lr=5e-5, weight_decay=0.01, max_grad_norm=1.0),
                       attack_detection=verify, gradient_verification=verify, quarantine=verify, param_integrity=verify, reassign=False)
    e = PipelineEngine(m, cfg, metrics=MetricsCollector())
    g = torch.Generator().manual_seed(0)
    bs = []
    for _ in range(2):
        ids = torch.randint(0, 50257, (8, 129), generator=g)
        bs.append({"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()})
    for i in range(14):
        e.train_step(bs[i % 2])
    e.flush()
    return [round(r["loss"], 5) for r in e.metrics.batch_metrics], e.attack_history
a, ha = run(True); b, hb = run(False)
print(a); print(b); print(len(ha), [ (h["step"], h["node_id"], h["attack_type"]) for h in ha][:10])
