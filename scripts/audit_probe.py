"""Per-check audit errors of a clean local run (which check of which stage would fail, and by how
much): wraps PipelineEngine._audit_one and prints (step, stage, kind bits, worst relative error)
plus the individual forward / dX / dW errors.  Usage:
  python scripts/audit_probe.py --model resnet50 --hw 224 --batch 64 --mbs 8 --nodes 8 --steps 4"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.models import get_model  # noqa: E402
from trustworthy_dl.parallel import pipeline as P  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--hw", type=int, default=224)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--mbs", type=int, default=8)
    ap.add_argument("--nodes", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--device", default="cuda:0" if torch.cuda.is_available() else "cpu")
    a = ap.parse_args()
    orig = P.PipelineEngine._audit_one
    rows = []

    def probe(self, st, x, m, M, y_seen=None, dy=None, labels=None, dx_seen=None, run=None, whash=None):
        from trustworthy_dl.security.grad_audit import sketch_mismatch
        flag, kind, err = orig(self, st, x, m, M, y_seen=y_seen, dy=dy, labels=labels, dx_seen=dx_seen, run=run,
                               whash=whash)
        bwd = self.cfg.audit_backward and (st.computes_loss or dy is not None)
        y_ref, dx_ref, sk_ref = self._recompute(st, x, dy, labels, M, backward=bwd)
        ef = self._audit_verdict(y_seen, y_ref)[1].item() if y_seen is not None and not st.computes_loss else None
        ed = self._audit_verdict(dx_seen, dx_ref)[1].item() if dx_seen is not None and dx_ref is not None else None
        ew = None
        if run is not None and sk_ref is not None:
            floor = 1e-3 * (run[1:] - run[:-1]).abs().amax()
            ew = sketch_mismatch(run[m + 1] - run[m], sk_ref, self.cfg.audit_grad_tol, floor)[1].item()
        rows.append((self.global_step, st.stage_id, int(kind.item()), round(err.item(), 5), ef, ed, ew))
        print(rows[-1], flush=True)
        return flag, kind, err
    P.PipelineEngine._audit_one = probe
    kw = {"num_classes": 1000} if a.model.startswith(("resnet50", "resnet18", "resnet34", "resnet101")) else {}
    m = get_model(a.model, seed=1, **kw)
    eng = P.PipelineEngine(m, P.EngineConfig(num_nodes=a.nodes, micro_batches=a.batch // a.mbs, device=a.device,
                                             monitor_seed=0, reassign=False, audit_targeted=False))
    g = torch.Generator().manual_seed(0)
    for _ in range(a.steps):
        x = torch.randn(a.batch, 3, a.hw, a.hw, generator=g)
        y = torch.randint(0, 10, (a.batch,), generator=g)
        eng.train_step({"input": x, "target": y})
    eng.flush()
    print("blamed", sorted({(r["step"], r["node_id"], r["attack_type"], r["audit_kind"]) for r in eng.attack_history}))


if __name__ == "__main__":
    main()
