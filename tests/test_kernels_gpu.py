"""Numerics of every native HIP kernel against a plain PyTorch fp32 reference (GPU only)."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.fixture(autouse=True)
def _native():
    from trustworthy_dl.ops import _lib
    _lib.lib()  # must load: no silent fallback
    torch.manual_seed(0)


@pytest.mark.parametrize("N", [768, 1024, 300])
def test_layernorm(N):
    from trustworthy_dl.ops import layer_norm
    M = 257
    x = torch.randn(M, N, device=DEV).bfloat16().requires_grad_(True)
    w = (1 + 0.1 * torch.randn(N, device=DEV)).bfloat16().requires_grad_(True)
    b = (0.1 * torch.randn(N, device=DEV)).bfloat16().requires_grad_(True)
    y = layer_norm(x, w, b, 1e-5)
    g = torch.randn_like(y)
    y.backward(g)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (N,), wr, br, 1e-5)
    yr.backward(g.float())
    assert _rel(y, yr) < 1e-2
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2
    assert _rel(b.grad, br.grad) < 2e-2


def test_linear_gelu_and_main_grad():
    from trustworthy_dl.ops import linear
    M, K, N = 512, 256, 1024
    x = torch.randn(M, K, device=DEV).bfloat16().requires_grad_(True)
    W = (torch.randn(K, N, device=DEV) * 0.05).bfloat16().requires_grad_(True)
    b = (torch.randn(N, device=DEV) * 0.1).bfloat16().requires_grad_(True)
    W.main_grad = torch.zeros(K, N, device=DEV)
    b.main_grad = torch.zeros(N, device=DEV)
    for act in ("gelu", None):
        W.main_grad.zero_()
        b.main_grad.zero_()
        x.grad = None
        y = linear(x, W, b, act)
        g = torch.randn_like(y)
        y.backward(g)
        xr, Wr, br = (t.detach().float().requires_grad_(True) for t in (x, W, b))
        yr = xr @ Wr + br
        if act == "gelu":
            yr = torch.nn.functional.gelu(yr, approximate="tanh")
        yr.backward(g.float())
        assert _rel(y, yr) < 1e-2, act
        assert _rel(x.grad, xr.grad) < 2e-2, act
        assert _rel(W.main_grad, Wr.grad) < 2e-2, act
        assert _rel(b.main_grad, br.grad) < 2e-2, act
        assert W.grad is None and b.grad is None


def test_linear_t():
    from trustworthy_dl.ops.layers import linear_t
    M, K, N = 384, 128, 640
    x = torch.randn(M, K, device=DEV).bfloat16().requires_grad_(True)
    W = (torch.randn(N, K, device=DEV) * 0.05).bfloat16().requires_grad_(True)
    y = linear_t(x, W)
    g = torch.randn_like(y)
    y.backward(g)
    xr, Wr = x.detach().float().requires_grad_(True), W.detach().float().requires_grad_(True)
    (xr @ Wr.t()).backward(g.float())
    assert _rel(y, xr @ Wr.t()) < 1e-2
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(W.grad, Wr.grad) < 2e-2


@pytest.mark.parametrize("T,H", [(128, 2), (256, 4), (384, 3)])
def test_flash_attention(T, H):
    from trustworthy_dl.ops import causal_attention
    B, D = 2, 64
    qkv = (torch.randn(B, T, 3 * H * D, device=DEV)).bfloat16().requires_grad_(True)
    o = causal_attention(qkv, H, True)
    g = torch.randn_like(o)
    o.backward(g)
    x = qkv.detach().float().requires_grad_(True)
    q, k, v = x.view(B, T, 3, H, D).permute(2, 0, 3, 1, 4)
    ref = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True)
    ref = ref.transpose(1, 2).reshape(B, T, H * D)
    ref.backward(g.float())
    assert _rel(o, ref) < 2e-2
    assert _rel(qkv.grad, x.grad) < 3e-2


def test_flash_attention_production_shape():
    """The benched GPT-2-medium shape (H = 16, T = 1024, causal) at B = 4 against fp32 SDPA, per
    gradient slice (dQ, dK, dV) with a relative Frobenius tolerance."""
    from trustworthy_dl.ops import causal_attention
    torch.manual_seed(1)
    B, T, H, D = 4, 1024, 16, 64
    qkv = (torch.randn(B, T, 3 * H * D, device=DEV)).bfloat16().requires_grad_(True)
    o = causal_attention(qkv, H, True)
    g = torch.randn_like(o)
    o.backward(g)
    x = qkv.detach().float().requires_grad_(True)
    q, k, v = x.view(B, T, 3, H, D).permute(2, 0, 3, 1, 4)
    ref = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, T, H * D)
    ref.backward(g.float())
    fro = lambda a, b: float((a.float() - b).norm() / b.norm())  # noqa: E731
    assert fro(o, ref) < 1e-2
    gq, gr = qkv.grad.view(B, T, 3, H * D), x.grad.view(B, T, 3, H * D)
    for i, name in enumerate("qkv"):
        assert fro(gq[:, :, i], gr[:, :, i]) < 2e-2, name


@pytest.mark.parametrize("B,T,H", [(2, 256, 4), (4, 1024, 16)])
def test_attention_bwd_fused_bias_grad(B, T, H):
    """The qkv bias gradient accumulated inside the attention backward kernels equals the fp64
    column sums of the bf16 gradient they return (every column, both causal and full)."""
    from trustworthy_dl.ops.layers import attn_bwd, attn_fwd
    torch.manual_seed(2)
    D = 64
    for causal in (True, False):
        qkv = torch.randn(B, T, 3 * H * D, device=DEV).bfloat16()
        out, lse, scale = attn_fwd(qkv, H, causal)
        dout = torch.randn_like(out)
        acc = torch.randn(3 * H * D, device=DEV)
        acc0 = acc.clone()
        dq = attn_bwd(qkv, out, lse, dout, H, causal, scale, bias_acc=acc)
        dq_plain = attn_bwd(qkv, out, lse, dout, H, causal, scale)
        assert torch.equal(dq, dq_plain)
        ref = acc0.double() + dq.double().reshape(-1, 3 * H * D).sum(0)
        err = float((acc.double() - ref).abs().max() / ref.abs().max())
        assert err < 1e-5, (causal, err)


def test_attention_rescale_branch():
    """Force the online-softmax running max to jump inside a row (rule 26)."""
    from trustworthy_dl.ops import causal_attention
    B, T, H, D = 1, 256, 1, 64
    qkv = torch.randn(B, T, 3 * H * D, device=DEV) * 0.1
    qkv[0, 200, 64:128] = 3.0   # a late key with a huge score for every query
    qkv[0, :, 0:64] = 3.0 / 8
    qkv = qkv.bfloat16()
    o = causal_attention(qkv, H, True)
    x = qkv.float()
    q, k, v = x.view(B, T, 3, H, D).permute(2, 0, 3, 1, 4)
    ref = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, T, H * D)
    assert _rel(o, ref) < 2e-2


@pytest.mark.parametrize("Hd", [256, 1024, 192])
def test_embedding(Hd):
    from trustworthy_dl.ops import embedding
    B, T, V = 2, 128, 1000
    ids = torch.randint(0, V, (B, T), device=DEV)
    ids[0, :5] = 7  # repeated ids collide in the scatter
    wte = torch.randn(V, Hd, device=DEV).bfloat16().requires_grad_(True)
    wpe = torch.randn(T, Hd, device=DEV).bfloat16().requires_grad_(True)
    y = embedding(ids, wte, wpe)
    g = torch.randn_like(y)
    y.backward(g)
    wr, pr = wte.detach().float().requires_grad_(True), wpe.detach().float().requires_grad_(True)
    yr = wr[ids] + pr[:T]
    yr.backward(g.float())
    assert _rel(y, yr) < 1e-2
    assert _rel(wte.grad, wr.grad) < 2e-2
    assert _rel(wpe.grad, pr.grad) < 2e-2


def test_cross_entropy_padded_vocab():
    from trustworthy_dl.ops import cross_entropy
    M, V, ld = 64, 1000, 1024
    logits = torch.randn(M, ld, device=DEV).bfloat16().requires_grad_(True)
    lr = logits.detach().float()[:, :V].clone().requires_grad_(True)  # before: backward reuses the buffer
    labels = torch.randint(0, V, (M,), device=DEV)
    loss = cross_entropy(logits, labels, V)
    loss.backward()
    ref = torch.nn.functional.cross_entropy(lr, labels)
    ref.backward()
    assert abs(float(loss) - float(ref)) < 1e-2
    assert _rel(logits.grad[:, :V], lr.grad) < 2e-2
    assert float(logits.grad[:, V:].abs().max()) == 0.0


def test_adamw_flat_matches_torch():
    from trustworthy_dl.parallel.flat import AdamWConfig, FlatParams
    m = torch.nn.Linear(64, 32)
    ref = torch.nn.Linear(64, 32)
    ref.load_state_dict(m.state_dict())
    fp = FlatParams(m.to(DEV), DEV, torch.float32)
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.0)
    cfg = AdamWConfig(lr=1e-2, weight_decay=0.0)
    for _ in range(3):
        g = torch.randn(fp.numel)
        fp.grad.copy_(g.to(DEV))
        off = 0
        for p, q in zip(fp.params, ref.parameters()):
            pass
        # map flat grads onto the reference params by name
        names = dict(ref.named_parameters())
        for i, n in enumerate(fp.names):
            names[n].grad = g[fp.offsets[i]:fp.offsets[i + 1]].view(fp.shapes[i]).clone()
        fp.adamw_step(cfg)
        opt.step()
    names = dict(ref.named_parameters())
    for i, n in enumerate(fp.names):
        assert torch.allclose(fp.view(fp.master, i).cpu(), names[n].detach(), atol=1e-5)


def test_adamw_skip_flag():
    from trustworthy_dl.parallel.flat import AdamWConfig, FlatParams
    m = torch.nn.Linear(16, 16).to(DEV)
    fp = FlatParams(m, DEV, torch.bfloat16)
    before = fp.master.clone()
    fp.grad.fill_(1.0)
    ctrl = torch.tensor([1.0, 1.0], device=DEV)
    fp.adamw_step(AdamWConfig(lr=1e-1), ctrl=ctrl)
    assert torch.equal(fp.master, before)
    assert float(fp.grad.abs().max()) == 0.0


def test_tensor_stats():
    from trustworthy_dl.ops.stats import tensor_stats
    from trustworthy_dl.security.attack_detection import numpy_tensor_statistics, TENSOR_STATS
    x = torch.randn(1 << 20, device=DEV) * 2 + 0.5
    x[::1000] += 5.0
    for dt in (torch.float32, torch.bfloat16):
        xt = x.to(dt)
        v = tensor_stats(xt).cpu()
        ref = numpy_tensor_statistics(xt.float().cpu().numpy())
        rng = ref["max"] - ref["min"]
        for i, k in enumerate(TENSOR_STATS):
            tol = rng / 2048 * 1.5 if k in ("median", "percentile_25", "percentile_75") else \
                1e-3 * max(1.0, abs(ref[k]))
            assert abs(float(v[i]) - ref[k]) <= tol, (dt, k, float(v[i]), ref[k])
        assert float(v[12]) == 0.0
    y = x.clone()
    y[3] = float("nan")
    assert float(tensor_stats(y)[12]) == 1.0


def test_grad_stats_matches_cpu():
    from trustworthy_dl.ops.stats import FlatGradStats
    sizes = [1000, 70000, 5, 40000]
    n = sum(sizes)
    gpu = FlatGradStats(sizes, DEV)
    cpu = FlatGradStats(sizes, "cpu")
    for step in range(3):
        g = torch.randn(n)
        a = gpu.compute(g.to(DEV)).cpu()
        b = cpu.compute(g.clone())
        # moments, norms, cosines
        for i in list(range(4)) + [5, 6, 9, 10, 11, 12, 13, 14, 15, 16, 17]:
            assert abs(float(a[i]) - float(b[i])) <= 2e-3 * max(1.0, abs(float(b[i]))), (step, i, a[i], b[i])
        assert torch.allclose(a[18:], b[18:], rtol=1e-3, atol=1e-4)


def test_grad_stats_offset_and_outlier_match_cpu():
    """The partial pass sums shifted powers about one per-chunk shift: a large common offset and a
    huge outlier at a chunk's first element must not cost the moments their precision."""
    from trustworthy_dl.ops.stats import CHUNK, FlatGradStats
    sizes = [5 * CHUNK + 33, 4 * CHUNK]
    n = sum(sizes)
    torch.manual_seed(11)
    for case in ("offset", "outlier"):
        g = torch.randn(n, dtype=torch.float64) * 0.01
        if case == "offset":
            g += 3.0
        else:
            g[CHUNK] = 1e3
            g[sizes[0]] = -5e2
        g = g.float()
        a = FlatGradStats(sizes, DEV).compute(g.to(DEV)).cpu()
        b = FlatGradStats(sizes, "cpu").compute(g.clone())
        for i in list(range(4)) + [5, 6, 9, 10, 11, 12, 13, 14, 15, 17]:
            assert abs(float(a[i]) - float(b[i])) <= 2e-3 * max(1.0, abs(float(b[i]))), (case, i, a[i], b[i])
        assert torch.allclose(a[18:18 + len(sizes)], b[18:18 + len(sizes)], rtol=1e-3, atol=1e-4)


def test_grad_stats_in_pieces_match_one_pass():
    """Partial passes over arbitrary chunk ranges (the per-layer overlap path) + the final stages
    give the single pass's result; the bare clipping sum of squares matches torch."""
    from trustworthy_dl.ops.stats import CHUNK, FlatGradStats, FlatSumSq
    sizes = [3 * CHUNK + 17, 5, 2 * CHUNK, 70000, 1]
    n = sum(sizes)
    a, b = FlatGradStats(sizes, DEV), FlatGradStats(sizes, DEV)
    for step in range(3):
        g = torch.randn(n, device=DEV)
        g[123] = float("inf") if step == 2 else g[123]
        ra = a.compute(g).clone()
        lo, hi = b.chunk_range_of(1, 4)
        b.partial(g, lo, hi)               # segments 1..3 early, the rest in compute()
        rb = b.compute(g).clone()
        assert torch.allclose(ra, rb, rtol=1e-6, atol=1e-7, equal_nan=True), (step, ra, rb)
    w = torch.tensor([1.0, 0.0, 1.0, 0.5, 1.0], device=DEV)
    g = torch.randn(n, device=DEV)
    sq = FlatSumSq(sizes, DEV).compute(g, w)
    ref = sum(float(wi) * float((x * x).sum()) for wi, x in zip(w, torch.split(g, sizes)))
    assert float(sq) == pytest.approx(ref, rel=1e-5)


def test_grad_stats_reduce_partial_bit_identical():
    """Split-K slabs reduced into the flat gradient AND its segment's partial statistics in one
    kernel == tdl_splitk_reduce_add followed by the plain partial pass: the same stored gradient and
    the same final statistics, bit for bit (one segment fused, the others plain)."""
    from trustworthy_dl.ops import _lib
    from trustworthy_dl.ops._lib import ptr, stream_ptr
    from trustworthy_dl.ops.stats import FlatGradStats
    torch.manual_seed(3)
    sizes = [1000, 3 * 65536 + 8, 4096, 77, 65536 * 2]
    g0 = torch.randn(sum(sizes), device=DEV)
    seg = 1
    off = sum(sizes[:seg])
    S = 4
    slabs = torch.randn(S, sizes[seg], device=DEV)
    outs = []
    for fused in (False, True):
        gs = FlatGradStats(sizes, DEV)
        for step in range(2):                 # the second step exercises the EMA reference
            g = g0.clone() * (1 + step)
            if fused:
                assert gs.reduce_partial(g, seg, slabs, S)
            else:
                _lib.call("tdl_splitk_reduce_add", ptr(g[off:off + sizes[seg]]), ptr(slabs), S, sizes[seg],
                          stream_ptr(g.device))
                c0, c1 = gs.chunk_range_of(seg, seg + 1)
                gs.partial(g, c0, c1)
            out = gs.compute(g).clone()
        outs.append((g, out, gs.ref.clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1]), (outs[0][1] - outs[1][1]).abs().max()
    assert torch.equal(outs[0][2], outs[1][2])


@pytest.mark.parametrize("kw", [{}, {"robust": "detrend", "window": 32},
                                {"robust": "detrend", "agg": "max", "abs_floor": 0.02, "rel_floor": 0.0,
                                 "z_decision": 8.0, "max_quarantine": 5},
                                {"robust": "detrend", "agg": "max", "abs_floor": 0.02, "rel_floor": 0.0,
                                 "z_decision": 8.0, "max_quarantine": 5, "early_gate": True}])
def test_zscore_matches_cpu(kw):
    from trustworthy_dl.ops.stats import DeviceZScore
    K = 17
    dg = DeviceZScore(K, DEV, history=50, warmup=10, **kw)
    dc = DeviceZScore(K, "cpu", history=50, warmup=10, **kw)
    g = torch.Generator().manual_seed(1)
    drift = torch.linspace(0, 3, K)
    for step in range(80):
        cur = torch.randn(K, generator=g) + drift * step / 20.0
        if step in (9, 30, 31, 60):   # step 9: inside the warm-up (10), after 8 entries: early gate
            cur = cur * 20
        a = dg.observe(cur.to(DEV)).cpu()
        b = dc.observe(cur.clone())
        assert float(a[0]) == float(b[0]), step
        if kw.get("early_gate") and step == 9:
            assert float(a[0]) == 1.0           # gross outlier flagged and kept out of the baseline
        assert abs(float(a[1]) - float(b[1])) < 1e-3 * max(1, float(b[1])), step


def test_trust_update_matches_python():
    from trustworthy_dl.core.trust_manager import STATUS_CODES, TrustManager
    from trustworthy_dl.ops.stats import trust_update
    N = 5
    tm = TrustManager(N, 0.7, decay_clock="step")
    vals = torch.ones(N, device=DEV)
    cnt = torch.zeros(N, dtype=torch.int32, device=DEV)
    st = torch.zeros(N, dtype=torch.int32, device=DEV)
    w = torch.tensor(tm.weights_vector(), device=DEV)
    g = torch.Generator().manual_seed(0)
    for step in range(40):
        tm.advance_step()
        met = torch.rand(N, 6, generator=g)
        met[:, 1] = 1 - met[:, 1] * 0.5
        flags = torch.zeros(N, dtype=torch.int32)
        if step == 10:
            flags[2] = 1
            tm.mark_compromised(2)
        for i in range(N):
            tm.update_trust_score(i, float(met[i, 0]), float(met[i, 1]), communication_latency=float(met[i, 2]),
                                  resource_utilization=float(met[i, 3]), error_rate=float(met[i, 4]),
                                  uptime=float(met[i, 5]))
        trust_update(vals, cnt, st, met.to(DEV), w, 0.7, tm.decay_rate, 1.0, flags.to(DEV), None)
        for i in range(N):
            assert abs(float(vals[i]) - tm.get_trust_score(i)) < 1e-5, (step, i)
            assert int(st[i]) == STATUS_CODES[tm.get_node_status(i)], (step, i)


def test_attack_inject_modes():
    from trustworthy_dl.ops.attack import AttackMode, inject_
    x = torch.randn(10001, device=DEV)
    y = x.clone()
    inject_(y, AttackMode.SCALE, 10.0)
    assert torch.allclose(y, x * 10)
    y = x.clone()
    inject_(y, AttackMode.SIGN_FLIP, 1.0)
    assert torch.allclose(y, -x)
    y = x.clone()
    inject_(y, AttackMode.NOISE, 1.0, seed=3, offset=7)
    z = x.clone()
    inject_(z, AttackMode.NOISE, 1.0, seed=3, offset=7)
    assert torch.equal(y, z)  # deterministic
    d = (y - x)
    assert abs(float(d.mean())) < 0.05 and abs(float(d.std()) - 1.0) < 0.05
    yb = x.bfloat16()
    inject_(yb, AttackMode.ZERO, 0.0)
    assert float(yb.float().abs().max()) == 0.0


def test_gpt2_engine_step_matches_cpu():
    """A GPT-2-tiny pipeline step on the GPU (bf16 native kernels) tracks the CPU fp32 reference."""
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    torch.manual_seed(0)
    ids = torch.randint(0, 50257, (4, 129))
    batch = {"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()}
    from trustworthy_dl.utils.metrics import MetricsCollector
    losses = {}
    for dev in ("cpu", "cuda:0"):
        m = get_model("gpt2-tiny", seq_len=128, seed=3)
        eng = PipelineEngine(m, EngineConfig(num_nodes=2, micro_batches=2, seq_len=128, device=dev),
                             metrics=MetricsCollector())
        for _ in range(4):
            eng.train_step(batch)
        eng.flush()
        losses[dev] = [r["loss"] for r in eng.metrics.batch_metrics]
    # every step, bf16 native kernels vs fp32 op-by-op reference (was: last step within 5 %)
    assert len(losses["cpu"]) == len(losses["cuda:0"]) == 4
    for a, b in zip(losses["cuda:0"], losses["cpu"]):
        assert abs(a - b) < 5e-3 * b, losses


@pytest.mark.parametrize("M,N", [(512, 1024), (32768, 4096)])
def test_bias_gelu_kernels_production_shape(M, N):
    """tdl_bias_gelu_fwd / _bwd (+ bias-gradient column sums) at GPT-2-medium's MLP shape
    (32 sequences x 1024 tokens, 4096 wide) against fp32 torch."""
    import torch.nn.functional as F
    from trustworthy_dl.ops import block
    torch.manual_seed(0)
    pre = (torch.randn(M, N, device=DEV) * 2).bfloat16()
    b = (torch.randn(N, device=DEV) * 0.5).bfloat16()
    f = block._bias_gelu_fwd(pre, b)
    u = (pre.float() + b.float()).requires_grad_(True)
    ref = F.gelu(u, approximate="tanh")
    assert _rel(f, ref) < 1e-2
    df = torch.randn(M, N, device=DEV).bfloat16()
    db = torch.zeros(N, device=DEV)
    dpre = block._bias_gelu_bwd(df, pre, b, db)
    (g,) = torch.autograd.grad(ref, u, df.float())
    assert _rel(dpre, g) < 1e-2
    assert float((db - g.sum(0)).norm() / g.sum(0).norm()) < 1e-3


def test_gpt2_half_block_stages_match_block_stages_on_gpu():
    """Stage boundaries inside blocks (unpaired attention / MLP halves, bf16 native kernels) give
    the same training trajectory as whole-block stages."""
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    torch.manual_seed(0)
    ids = torch.randint(0, 50257, (4, 129))
    batch = {"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()}
    losses = {}
    for g in ("block", "half"):
        m = get_model("gpt2-mini", seq_len=128, seed=3)
        eng = PipelineEngine(m, EngineConfig(num_nodes=4, micro_batches=2, seq_len=128, device="cuda:0",
                                             layer_granularity=g, reassign=False))
        if g == "half":
            assert any((b - a) % 2 for a, b in eng.plan.ranges[1:-1]), eng.plan.ranges
        for _ in range(4):
            eng.train_step(batch)
        eng.flush()
        losses[g] = eng.last_loss
    assert abs(losses["block"] - losses["half"]) < 0.02 * losses["block"], losses


@pytest.mark.parametrize("N", [1024, 768])
def test_add_bias_ln_and_residual_ln_bwd(N):
    """tdl_add_bias_ln_fwd and the residual/colsum variant of LN backward vs fp32 torch."""
    from trustworthy_dl.ops.block import _add_bias_ln_fwd, _ln_bwd
    M = 1000
    bf = lambda *s, sc=1.0: (sc * torch.randn(*s, device=DEV)).bfloat16()
    x, z, dres, dy = bf(M, N), bf(M, N), bf(M, N), bf(M, N)
    bz, b2, bb = bf(N, sc=0.1), bf(N, sc=0.1), bf(N, sc=0.1)
    w = (1 + 0.1 * torch.randn(N, device=DEV)).bfloat16()
    y1, y1b, h, mean, rstd = _add_bias_ln_fwd(x, z, bz, b2, w, bb, 1e-5)
    y1r = x.float() + z.float() + bz.float()
    assert _rel(y1, y1r) < 1e-2
    assert _rel(y1b, y1r + b2.float()) < 1e-2
    hr = torch.nn.functional.layer_norm(y1.float(), (N,), w.float(), bb.float(), 1e-5)
    assert _rel(h, hr) < 1e-2
    acc = [torch.zeros(N, device=DEV) for _ in range(4)]
    dx = _ln_bwd(dy, y1, w, mean, rstd, acc[0], acc[1], dres=dres, sres_acc=acc[2], sdx_acc=acc[3])
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (y1, w, bb))
    torch.nn.functional.layer_norm(xr, (N,), wr, br, 1e-5).backward(dy.float())
    assert _rel(dx, xr.grad + dres.float()) < 2e-2
    assert _rel(acc[0], wr.grad) < 2e-2
    assert _rel(acc[1], br.grad) < 2e-2
    assert _rel(acc[2], dres.float().sum(0)) < 1e-3
    assert _rel(acc[3], dx.float().sum(0)) < 1e-3


def test_fused_gpt2_block_matches_fp32():
    """Fused single-node block (bf16, native kernels, main_grad accumulation) vs the fp32 CPU
    op-by-op module on the same weights."""
    import copy
    from trustworthy_dl.models.gpt2 import GPT2Config, GPT2Block
    cfg = GPT2Config(n_embd=256, n_head=4, n_layer=1)
    ref = GPT2Block(cfg)
    for p in ref.parameters():
        torch.nn.init.normal_(p, std=0.05)
    ref.fused = False
    blk = copy.deepcopy(ref).to(DEV).bfloat16()
    blk.fused = True
    for p in blk.parameters():
        p.main_grad = torch.zeros(p.shape, device=DEV)
    x = torch.randn(2, 256, 256)
    g = torch.randn(2, 256, 256)
    xr = x.clone().requires_grad_(True)
    ref(xr).backward(g)
    xd = x.to(DEV).bfloat16().requires_grad_(True)
    yd = blk(xd)
    yd.backward(g.to(DEV).bfloat16())
    yr = ref(x)
    assert _rel(yd.cpu(), yr) < 2e-2
    assert _rel(xd.grad.cpu(), xr.grad) < 3e-2
    for (n, p), (_, q) in zip(blk.named_parameters(), ref.named_parameters()):
        assert p.grad is None, n
        assert _rel(p.main_grad.cpu(), q.grad) < 3e-2, n


@pytest.mark.gpu
def test_fused_gpt2_block_production_shape_matches_fp32():
    """The benched block shape (GPT-2-medium: width 1024, 16 heads, T = 1024; B = 2) with the
    default GEMM routing, fused bf16 forward + backward vs the fp32 CPU op-by-op module: output, dx
    and every parameter's fp32 main_grad."""
    import copy
    from trustworthy_dl.models.gpt2 import GPT2Config, GPT2Block
    torch.manual_seed(0)
    cfg = GPT2Config(n_embd=1024, n_head=16, n_layer=1)
    ref = GPT2Block(cfg)
    for p in ref.parameters():
        torch.nn.init.normal_(p, std=0.02)
    ref.fused = False
    blk = copy.deepcopy(ref).to(DEV).bfloat16()
    blk.fused = True
    for p in blk.parameters():
        p.main_grad = torch.zeros(p.shape, device=DEV)
    x = torch.randn(2, 1024, 1024)
    g = torch.randn(2, 1024, 1024)
    xr = x.clone().requires_grad_(True)
    yr = ref(xr)
    yr.backward(g)
    xd = x.to(DEV).bfloat16().requires_grad_(True)
    yd = blk(xd)
    yd.backward(g.to(DEV).bfloat16())
    assert _rel(yd.float().cpu(), yr.detach()) < 2e-2
    assert _rel(xd.grad.float().cpu(), xr.grad) < 3e-2
    for (n, p), (_, q) in zip(blk.named_parameters(), ref.named_parameters()):
        assert p.grad is None, n
        assert _rel(p.main_grad.cpu(), q.grad) < 3e-2, n


@pytest.mark.gpu
@pytest.mark.parametrize("M,K,N", [(65536, 1024, 3072), (65536, 1024, 1024), (65536, 1024, 4096),
                                   (65536, 4096, 1024), (8192, 1024, 1024), (4096, 1000, 264)])
def test_wgrad_native_accumulates(M, K, N):
    """Weight-gradient products (x^T dy into an fp32 main_grad) on the native persistent kernel at
    the GPT-2-medium production shapes (64k tokens: qkv / out-proj / fc / proj), a short token count
    and a ragged width, against fp32 torch."""
    from trustworthy_dl.ops import gemm
    from trustworthy_dl.ops.layers import wgrad_acc
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    acc = torch.randn(K, N, device="cuda")
    ref = acc + x.float().t() @ dy.float()
    if K % 8 == 0 and N % 8 == 0:
        assert gemm.supported(x.t(), dy)
    if M == 65536:
        assert gemm.wgrad_split(M, K, N) > 1
    wgrad_acc(acc, x.t(), dy)
    assert float((acc - ref).norm() / ref.norm()) < 1e-3


@pytest.mark.gpu
def test_weight_checksum_deterministic_and_sensitive():
    from trustworthy_dl.ops.stats import checksum
    x = torch.randn(3_000_001, device="cuda").to(torch.bfloat16)
    a, b = checksum(x).clone(), checksum(x).clone()
    assert torch.equal(a, b)  # bit-identical on identical data
    v = x.double().cpu()
    w = (torch.arange(v.numel(), dtype=torch.float64) % 1021) + 1
    ref = torch.stack([v.sum(), (v * v).sum(), (v * w).sum()])
    assert torch.allclose(a.cpu(), ref, rtol=1e-9, atol=1e-6)
    y = x.clone()
    y[1_234_567] = (y[1_234_567].float() * 1.01).to(torch.bfloat16)  # one weight nudged
    assert not torch.equal(checksum(y), a)


@pytest.mark.parametrize("chunk", [None, 96])
def test_fused_lm_head_cross_entropy_matches_fp32(chunk):
    """Tied LM head + CE as one node (tdl_xent_fused, optional logits chunking) vs fp32 torch:
    loss, dX, dW (plain grad and main_grad accumulation), ignored labels, padded vocab."""
    from trustworthy_dl.ops.layers import lm_head_cross_entropy
    torch.manual_seed(0)
    N, n, V, Vp = 300, 128, 1000, 1024
    x = (torch.randn(N, n, device=DEV) * 0.5).bfloat16().requires_grad_(True)
    w = (torch.randn(Vp, n, device=DEV) * 0.05).bfloat16()
    w[V:] = 0
    w.requires_grad_(True)
    labels = torch.randint(0, V, (N,), device=DEV)
    labels[::7] = -100
    seen = []
    loss = lm_head_cross_entropy(x, w, labels, V, observe=lambda t: seen.append(t.float().clone()),
                                 chunk_rows=chunk)
    (loss * 0.5).backward()
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    logits = xr @ wr.t()
    ref = torch.nn.functional.cross_entropy(logits[:, :V], labels, ignore_index=-100)
    (ref * 0.5).backward()
    assert abs(float(loss) - float(ref)) < 2e-3 * float(ref)
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2
    assert seen and _rel(seen[0], logits[: seen[0].shape[0]].detach()) < 1e-2
    # main_grad accumulation path
    w2 = w.detach().clone().requires_grad_(True)
    w2.main_grad = torch.zeros(Vp, n, device=DEV)
    x2 = x.detach().clone().requires_grad_(True)
    (lm_head_cross_entropy(x2, w2, labels, V, chunk_rows=chunk) * 0.5).backward()
    assert w2.grad is None
    assert _rel(w2.main_grad, wr.grad) < 2e-2


def test_lm_head_gpt2_vocab_native_dx_matches_fp32():
    """GPT-2 vocab (V = 50257 padded to 50304, ignored labels): dX runs on gemm_pd over the cached
    [n, Vp] copy of the tied weight (layers._lmhead_dx); loss / dX / dW vs fp32, and the copy is
    rebuilt after the weight changes (new weight generation)."""
    from trustworthy_dl.ops import gemm
    from trustworthy_dl.ops.layers import _lmhead_dx, bump_weight_generation, fwd_weight, lm_head_cross_entropy
    torch.manual_seed(3)
    N, n, V, Vp = 512, 1024, 50257, 50304
    x = (torch.randn(N, n, device=DEV) * 0.5).bfloat16().requires_grad_(True)
    w = (torch.randn(Vp, n, device=DEV) * 0.05).bfloat16()
    w[V:] = 0
    w.requires_grad_(True)
    labels = torch.randint(0, V, (N,), device=DEV)
    labels[::5] = -100
    assert gemm.supported(torch.empty(N, Vp, dtype=torch.bfloat16, device=DEV), fwd_weight(w.detach()))
    loss = lm_head_cross_entropy(x, w, labels, V)
    loss.backward()
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    ref = torch.nn.functional.cross_entropy((xr @ wr.t())[:, :V], labels, ignore_index=-100)
    ref.backward()
    assert abs(float(loss) - float(ref)) < 2e-3 * float(ref)
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 2e-2
    # the direct product and a changed weight (the cached transposed copy must follow it)
    dl = (torch.randn(N, Vp, device=DEV) * 1e-3).bfloat16()
    with torch.no_grad():
        assert _rel(_lmhead_dx(dl, w.detach()), dl.float() @ w.detach().float()) < 1e-2
        w2 = w.detach()
        w2.mul_(-1.0)
        bump_weight_generation()
        assert _rel(_lmhead_dx(dl, w2), dl.float() @ w2.float()) < 1e-2


@pytest.mark.parametrize("V,ld", [(50257, 50304), (32000, 32000), (1000, 1024)])
def test_xent_fused_rows_vs_fp32(V, ld):
    """tdl_xent_fused on full GPT-2-vocab rows, a 32k vocab and a small padded row: loss, lse and
    in-place dlogits vs fp32 (the default two-pass kernel; TDL_XENT_REG=1 runs the register one)."""
    from trustworthy_dl.ops import _lib
    from trustworthy_dl.ops._lib import ptr, stream_ptr
    torch.manual_seed(1)
    M = 64
    logits = (torch.randn(M, ld, device=DEV) * 3.0).bfloat16()
    labels = torch.randint(0, V, (M,), device=DEV)
    labels[::5] = -100
    ref_in = logits.float()[:, :V]
    loss = torch.empty(M, device=DEV)
    lse = torch.empty(M, device=DEV)
    n_valid = int((labels != -100).sum())
    scale = torch.tensor([1.0 / n_valid], device=DEV)
    buf = logits.clone()
    _lib.call("tdl_xent_fused", ptr(buf), ptr(labels), ptr(loss), ptr(lse), ptr(scale), M, V, ld,
              stream_ptr(buf.device))
    torch.cuda.synchronize()
    ref_lse = torch.logsumexp(ref_in, dim=1)
    assert torch.allclose(lse, ref_lse, rtol=1e-5, atol=1e-4)
    valid = labels != -100
    ref_loss = ref_lse - ref_in.gather(1, labels.clamp(min=0)[:, None])[:, 0]
    assert torch.allclose(loss[valid], ref_loss[valid], rtol=1e-4, atol=1e-3)
    assert torch.all(loss[~valid] == 0)
    p = torch.softmax(ref_in, dim=1)
    p[valid, labels[valid]] -= 1.0
    p[~valid] = 0
    ref_d = p / n_valid
    d = buf.float()
    assert _rel(d[:, :V], ref_d) < 1e-2
    assert torch.all(d[:, V:] == 0)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n", [2, 5, 16])
def test_cosine_gram_native_matches_torch(n, dtype):
    """K6: N x N cosine Gram of N flat vectors read in place (attack_detector.py:143-162)."""
    from trustworthy_dl.ops.stats import cosine_gram
    torch.manual_seed(n)
    base = torch.randn(300_001, device=DEV)
    xs = [(base * (i % 3 - 1 + 0.3) + torch.randn(300_001, device=DEV) * 0.5).to(dtype) for i in range(n)]
    g = cosine_gram(xs)
    X = torch.stack([x.double().cpu() for x in xs])
    ref = (X @ X.t()) / (X.norm(dim=1)[:, None] * X.norm(dim=1)[None, :])
    assert torch.allclose(g.double().cpu(), ref, atol=1e-5), (g, ref)
    assert torch.equal(cosine_gram(xs), g)   # deterministic


@pytest.mark.parametrize("features", ["targeted", "reference"])
def test_verifier_fused_tail_matches_torch_form(features, monkeypatch):
    """csrc/stats.hip verify_finish_kernel (one launch for the verifier's step tail) against the
    torch form it replaces, over 30 steps with clean, scaled, sign-flipped and non-finite
    gradients and anomalous outputs: same digests (flags exactly), same EMA baselines and
    quarantine control."""
    from trustworthy_dl.security import stage_verifier as sv
    sizes = [300, 1000, 64, 4096, 17]
    mk = lambda: sv.StageVerifier(sizes, "cuda", warmup=5, features=features, serialize_streams=True)  # noqa: E731
    A, B = mk(), mk()
    g = torch.Generator(device="cuda").manual_seed(0)
    base = torch.randn(sum(sizes), device="cuda", generator=g)
    for step in range(30):
        flat = base + 0.3 * torch.randn(sum(sizes), device="cuda", generator=g)
        if step in (12, 13):
            flat = -flat                      # sign flip
        if step == 17:
            flat = flat * 50.0                # scaled
        if step == 21:
            flat[5] = float("nan")            # non-finite
        y = torch.randn(4, 64, device="cuda", generator=g).bfloat16()
        if step in (15, 25):
            y = y * 20.0
        loss = torch.tensor(3.0 - 0.01 * step, device="cuda")
        hm = [0.1 * step, 0.5, 0.0, 1.0]
        outs = []
        for v, fused in ((A, True), (B, False)):
            monkeypatch.setattr(sv, "VERIFY_FUSED", fused)
            v.observe_output(y)
            outs.append(v.finish_step(flat, loss, hm, step in (12, 13, 17), 2).clone())
        da, db = outs
        for k in (sv.D_OUT_FLAG, sv.D_GRAD_FLAG, sv.D_PRESENT, sv.D_STAGE, sv.D_ATTACK_TRUTH):
            assert float(da[k]) == float(db[k]), (step, k, da.tolist(), db.tolist())
        fin = torch.isfinite(db)
        assert torch.equal(torch.isfinite(da), fin), step
        # z-scores / confidences: the features' logs round differently (logf in the kernel vs
        # torch.log), and a MAD-scaled z magnifies that; every other slot to fp32 rounding
        zs = [sv.D_OUT_Z, sv.D_GRAD_Z, sv.D_OUT_CONF, sv.D_GRAD_CONF]
        tight = fin.clone()
        tight[zs] = False
        assert torch.allclose(da[tight], db[tight], rtol=1e-4, atol=1e-5), (step, (da - db).abs().max())
        assert torch.allclose(da[zs], db[zs], rtol=2e-2, atol=1e-3), (step, da[zs].tolist(), db[zs].tolist())
        for x, y_ in ((A.out_mu, B.out_mu), (A.out_sd, B.out_sd), (A.out_n, B.out_n), (A.norm_n, B.norm_n),
                      (A.ctrl, B.ctrl)):
            assert torch.allclose(x, y_, rtol=1e-5, atol=1e-6), step
        fe = torch.isfinite(B.norm_ema)
        assert torch.allclose(A.norm_ema[fe], B.norm_ema[fe], rtol=1e-5, atol=1e-6), step


def test_flash_attention_long_sequence_dynamic_lds():
    """T = 12288: the dK/dV kernel stages lse / delta for 12288 queries in 96 KiB of dynamic LDS
    (past the 64 KiB default, raised at launch); gradients vs fp32 SDPA."""
    from trustworthy_dl.ops import causal_attention
    torch.manual_seed(3)
    B, T, H, D = 1, 12288, 1, 64
    qkv = (torch.randn(B, T, 3 * H * D, device=DEV) * 0.5).bfloat16().requires_grad_(True)
    o = causal_attention(qkv, H, True)
    g = torch.randn_like(o)
    o.backward(g)
    x = qkv.detach().float().requires_grad_(True)
    q, k, v = x.view(B, T, 3, H, D).permute(2, 0, 3, 1, 4)
    ref = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2).reshape(B, T, H * D)
    ref.backward(g.float())
    assert _rel(o, ref) < 2e-2
    assert _rel(qkv.grad, x.grad) < 3e-2
