import os, sys, torch
sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import test_engine_gpu as T
res = {}
for mode in ["0", "1", "auto"]:
    os.environ["TDL_FUSED_GRAD_STATS"] = mode
    for ser in (False, True):
        eng, l, d, w = T._run(serialize_streams=ser, output_check="first")
        res[(mode, ser)] = d
        st = list(eng.stages.values())
        print(mode, ser, "loss", l, "side_ok", [getattr(s, "side_reduce_ok", None) for s in st], "audit", eng.cfg.audit, flush=True)
base = res[("0", True)]
for k, d in res.items():
    diff = (d - base).abs()
    idx = (diff > 1e-5).nonzero().tolist()
    print(k, "maxdiff", float(diff.max()), "idx", idx[:12], flush=True)
