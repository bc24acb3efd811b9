"""Per-step detector trace of one attack scenario (debug)."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.attacks.adversarial_attacks import AdversarialAttacker, AttackConfig
from trustworthy_dl.models import get_model
from trustworthy_dl.parallel.flat import AdamWConfig
from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
from trustworthy_dl.utils.data_loader import MarkovLanguageModeling
import trustworthy_dl.security.stage_verifier as SVm
scale = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
mode = sys.argv[3] if len(sys.argv) > 3 else "scale"
att = AdversarialAttacker(AttackConfig(attack_types=["gradient_poisoning"], gradient_mode=mode, gradient_scale=scale,
                                       target_nodes=[int(os.environ.get("DBG_TARGET", 4))],
                                       start_step=int(os.environ.get("DBG_START", 100)),
                                       probability=float(os.environ.get("DBG_P", 0.2)), seed=int(os.environ.get("DBG_SEED", 7))))
att.activate_attacks()
model = get_model("gpt2-medium", seq_len=1024, seed=11)
cfg = EngineConfig(num_nodes=8, micro_batches=int(os.environ.get("DBG_M", 2)), seq_len=1024, device="cuda:0",
                   reassign=os.environ.get("DBG_REASSIGN", "0") == "1",
                   adamw=AdamWConfig(lr=1e-4, weight_decay=0.01, max_grad_norm=1.0,
                                     warmup_steps=int(os.environ.get("DBG_WARMUP", 50))))
eng = PipelineEngine(model, cfg, attacker=att)
rows = []
orig = SVm.StageVerifier.finish_step
def fs(self, flat, loss, hm, truth, sid):
    d = orig(self, flat, loss, hm, truth, sid)
    if sid == int(os.environ.get("DBG_TARGET", 4)) and (truth or float(self.grad_det.out[0]) > 0):
        rows.append((eng.global_step, sid, int(truth), round(float(self.grad_stats.out[16]), 3), float(d[3]),
                     [round(float(x), 3) for x in self._grad_features(self.grad_stats.out)],
                     [round(float(x), 2) for x in self.grad_det.out[:2]], round(float(self.out_det.out[1]), 2)))
    return d
SVm.StageVerifier.finish_step = fs
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 141
for b in MarkovLanguageModeling(8, 1024, 8192, num_batches=steps, seed=0):
    eng.train_step(b)
eng.flush()
for r in rows:
    print(r)
print("hist", [(a["step"], a["node_id"], a["attack_type"]) for a in eng.attack_history][:60])
print("inj", [(i["step"], i["node"]) for i in att.injections][:20])
print("grace", eng.t_grace.tolist())
