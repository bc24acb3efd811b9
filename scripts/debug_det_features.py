"""Dump per-step detector features / z-scores of a clean GPT-2 run (debug for false positives)."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.models import get_model
from trustworthy_dl.parallel.flat import AdamWConfig
from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
from trustworthy_dl.utils.data_loader import MarkovLanguageModeling
import trustworthy_dl.security.stage_verifier as SVm

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 120
model = get_model("gpt2-medium", seq_len=1024, seed=11)
cfg = EngineConfig(num_nodes=8, micro_batches=2, seq_len=1024, device="cuda:0", reassign=False,
                   adamw=AdamWConfig(lr=1e-4, weight_decay=0.01, max_grad_norm=1.0), quarantine=False)
eng = PipelineEngine(model, cfg)
rows = []
orig = SVm.StageVerifier.finish_step
def fs(self, flat, loss, hm, truth, sid):
    d = orig(self, flat, loss, hm, truth, sid)
    if sid in (0, 1, 7):
        rows.append({"step": eng.global_step, "stage": sid, "out_feat": [round(float(x), 4) for x in self._out_features()],
                     "out_z": [round(float(x), 2) for x in self.out_det.out[:7]],
                     "grad_feat": [round(float(x), 4) for x in self._grad_features(self.grad_stats.out)],
                     "grad_z": [round(float(x), 2) for x in self.grad_det.out[:8]], "mon": eng._mon_idx})
    return d
SVm.StageVerifier.finish_step = fs
for b in MarkovLanguageModeling(8, 1024, 50257, num_batches=steps, seed=0):
    eng.train_step(b)
eng.flush()
for r in rows:
    print(json.dumps(r))
print(json.dumps({"flags": [(a["step"], a["node_id"], a["attack_type"]) for a in eng.attack_history][:40]}))
