"""Forward-layout weight copies (ops/block.py ``fwd_weight``): exact values, cached per weight
generation, rebuilt after torch in-place writes, after the native AdamW update (raw-pointer writes
that torch's version counter does not see) and never stale inside the engine."""
import os

import pytest
import torch

from trustworthy_dl.core.trust_manager import TrustManager
from trustworthy_dl.models import get_model
from trustworthy_dl.ops import block as B
from trustworthy_dl.parallel.flat import AdamWConfig
from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine

pytestmark = pytest.mark.gpu


def test_fwd_weight_exact_cached_and_refreshed():
    w = (torch.randn(256, 768, device="cuda") * 0.02).to(torch.bfloat16)
    a = B.fwd_weight(w)
    assert a.shape == w.shape and torch.equal(a, w)
    assert a.data_ptr() != w.data_ptr() and a.stride() == (1, 256)      # [out, in] storage
    assert B.fwd_weight(w).data_ptr() == a.data_ptr()                  # cached
    w.add_(1.0)                                                         # torch write: version bump
    assert torch.equal(B.fwd_weight(w), w)
    w.view(-1)[:10].fill_(3.0)                                          # write through a view
    assert torch.equal(B.fwd_weight(w), w)
    B.bump_weight_generation()                                          # raw writers bump the generation
    assert torch.equal(B.fwd_weight(w), w)


@pytest.mark.parametrize("R,C", [(1024, 3072), (4096, 1024), (64, 128), (192, 64)])
def test_native_transpose_matches_torch(R, C):
    from trustworthy_dl.ops import _lib
    from trustworthy_dl.ops._lib import ptr, stream_ptr
    w = torch.randn(R, C, device="cuda").to(torch.bfloat16)
    out = torch.empty(C, R, dtype=torch.bfloat16, device="cuda")
    _lib.call("tdl_transpose_bf16", ptr(w), ptr(out), R, C, stream_ptr(w.device))
    torch.cuda.synchronize()
    assert torch.equal(out, w.t())


def _batches(n, bs=8, T=128, seed=0):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        ids = torch.randint(0, 1024, (bs, T + 1), generator=g)
        out.append({"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()})
    return out


def test_engine_never_uses_stale_forward_weights(monkeypatch):
    m = get_model("gpt2-mini", seq_len=128, seed=0, vocab_size=1024)   # width 256: fused block
    cfg = EngineConfig(num_nodes=2, micro_batches=2, seq_len=128, device="cuda:0",
                       adamw=AdamWConfig(lr=1e-2), reassign=False)
    eng = PipelineEngine(m, cfg, TrustManager(2))
    batches = _batches(4)
    for b in batches[:3]:
        eng.train_step(b)
    eng.flush()
    cached = eng.eval_step(batches[3])                       # forward GEMMs on the [out, in] copies
    monkeypatch.setenv("TDL_FWD_WEIGHT_T", "0")
    direct = eng.eval_step(batches[3])                       # forward GEMMs on the parameters
    torch.cuda.synchronize()
    assert abs(cached - direct) <= 2e-3 * abs(direct), (cached, direct)
    # every cached copy equals its parameter after the last (native AdamW) update
    monkeypatch.setenv("TDL_FWD_WEIGHT_T", "1")
    eng.eval_step(batches[3])
    from trustworthy_dl.ops import layers as L
    n = 0
    for st in eng.stages.values():
        for p in st.module.parameters():
            c = getattr(p, "_tdl_fwd_t", None)
            if c is None:
                continue
            if c[0][0] == L._WEIGHT_GEN[0]:      # built for the current weights (this forward)
                assert torch.equal(c[1].t(), p.detach()), "stale forward-layout copy"
                n += 1
            else:   # the tied LM-head copy (built by the last backward's dX): refreshed on its next use
                with torch.no_grad():
                    assert torch.equal(B.fwd_weight(p), p.detach())
                assert p._tdl_fwd_t[0][0] == L._WEIGHT_GEN[0]
    assert n >= 4 * 4, n   # 4 blocks x 4 GEMM weights (+ the tied LM-head copy, prebuilt at the forward)


def test_prebuild_fwd_weights_batched_matches_lazy():
    """The batched rebuild (one tdl_transpose_bf16_batch launch per 64 weights, ops/layers.py
    prebuild_fwd_weights) refreshes exactly the stale copies fwd_weight built before, to the same
    values; weights without a copy, or with shapes the kernel does not take, are left to fwd_weight."""
    from trustworthy_dl.ops import layers as L
    shapes = [(1024, 3072), (1024, 1024), (4096, 1024), (64, 128)] * 20 + [(192, 64), (100, 64)]
    ws = [(torch.randn(*s, device="cuda") * 0.02).to(torch.bfloat16) for s in shapes]
    for w in ws[:-1]:
        B.fwd_weight(w)                  # lazily built copies (the 100 x 64 one never gets one)
    L.bump_weight_generation()
    for w in ws:
        w.mul_(-1.5)
    L.bump_weight_generation()
    L.prebuild_fwd_weights(ws)
    torch.cuda.synchronize()
    for w in ws[:-1]:
        key, wt = w._tdl_fwd_t
        assert key[0] == L._WEIGHT_GEN[0] and torch.equal(wt.t(), w)
        assert B.fwd_weight(w).data_ptr() == wt.data_ptr()   # cache hit: no rebuild
    assert getattr(ws[-1], "_tdl_fwd_t", None) is None
