"""Which hipBLASLt epilogue configurations have an algorithm on this GPU, and how fast (probe)."""
import json, os, statistics, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from trustworthy_dl.ops import blaslt, _lib, block

_lib.lib()
dev = torch.device("cuda:0")
M, C = 32768, 1024
N = 4 * C
r = lambda *s, sc=1.0: ((torch.rand(*s, device=dev) * 2 - 1) * sc).bfloat16()
h2, wfc, dy, wp = r(M, C), r(C, N, sc=0.05), r(M, C), r(N, C, sc=0.05)
wfc_t = wfc.t().contiguous()   # [N, C]
pre = torch.empty(M, N, dtype=torch.bfloat16, device=dev)


def timeit(fn, iters=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / iters)
    return statistics.median(ts)


for bdt in (torch.bfloat16, torch.float32):
    bias = r(N, sc=0.1).to(bdt)
    for name, opA, A, lda in (("NN", 0, wfc, N), ("TN", 1, wfc_t, C)):
        y = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        for epi_name, epi, aux in (("BIAS", 4, None), ("GELU_BIAS", 36, None), ("GELU_AUX_BIAS", 164, pre)):
            call = lambda: blaslt.gemm_colmajor(opA, 0, N, M, C, 1.0, A, lda, h2, C, 0.0, y, N, y, N, epi, bias, aux,
                                                N if aux is not None else 0)
            ok = call()
            rec = {"layout": name, "bias": str(bdt), "epi": epi_name, "supported": ok}
            if ok:
                rec["ms"] = round(timeit(call), 4)
            print(json.dumps(rec), flush=True)
# reference: torch.mm + separate GELU kernel, torch.mm alone
ref = lambda: block._bias_gelu_fwd(torch.mm(h2, wfc_t.t()), r(N).bfloat16() if False else bias.bfloat16())
print(json.dumps({"ref": "torch.mm(NT)+bias_gelu_fwd", "ms": round(timeit(lambda: block._bias_gelu_fwd(torch.mm(h2, wfc_t.t()), bias.bfloat16())), 4)}))
print(json.dumps({"ref": "torch.mm(NT)", "ms": round(timeit(lambda: torch.mm(h2, wfc_t.t())), 4)}))
# backward: DGELU_BGRAD
db = torch.zeros(N, device=dev)
d = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
for name, opA, A, lda in (("TN", 1, wp, C), ("NN", 0, wp.t().contiguous(), N)):
    for bdt in (torch.float32, torch.bfloat16):
        dbb = torch.zeros(N, device=dev, dtype=bdt)
        call = lambda: blaslt.gemm_colmajor(opA, 0, N, M, C, 1.0, A, lda, dy, C, 0.0, d, N, d, N, 208, dbb, pre, N)
        ok = call()
        rec = {"layout": name, "bgrad": str(bdt), "epi": "DGELU_BGRAD", "supported": ok}
        if ok:
            rec["ms"] = round(timeit(call), 4)
        print(json.dumps(rec), flush=True)
print(json.dumps({"ref": "torch.mm+bias_gelu_bwd", "ms": round(timeit(lambda: block._bias_gelu_bwd(torch.mm(dy, wp.t()), pre, bias.bfloat16(), db)), 4)}))
