"""Native MFMA GEMM (csrc/gemm.hip) vs a plain PyTorch fp32 reference of the same op (GPU only).

Covers the four operand storage forms (k-contiguous / row-contiguous for A and B), every fused
epilogue, ragged M and N (tile clamping + store masks), split-K slabs and atomics."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float(), b.float()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-20))


@pytest.fixture(autouse=True)
def _native():
    from trustworthy_dl.ops import _lib
    _lib.lib()
    torch.manual_seed(0)


def _rand(*shape, scale=1.0):
    return ((torch.rand(*shape, device=DEV) * 2 - 1) * scale).bfloat16()


def _view(t_logical, transposed):
    """Same logical matrix, stored row-major (False) or as a transposed view (True)."""
    return t_logical.t().contiguous().t() if transposed else t_logical.contiguous()


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("M,N,K", [(512, 256, 128), (768, 1024, 320), (520, 264, 64)])
def test_layouts(ta, tb, M, N, K):
    from trustworthy_dl.ops import gemm
    a = _view(_rand(M, K), ta)
    b = _view(_rand(K, N, scale=0.1), tb)
    out = gemm.matmul(a, b)
    ref = a.float() @ b.float()
    assert _rel(out, ref) < 1e-2, (ta, tb, M, N, K)


def test_bias_gelu_resadd_dgelu():
    from trustworthy_dl.ops import gemm
    M, N, K = 1000, 512, 256          # ragged M (1000 = 3 x 256 + 232)
    x = _rand(M, K)
    w = _rand(K, N, scale=0.1)
    bias = _rand(N, scale=0.5)
    ref_pre = x.float() @ w.float() + bias.float()
    # bias only
    y = gemm.matmul(x, w, bias=bias)
    assert _rel(y, ref_pre) < 1e-2
    # bias + gelu (pre-activation stored too)
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    f = gemm.matmul(x, w, bias=bias, epi="gelu", aux=pre)
    assert _rel(pre, ref_pre) < 1e-2
    assert _rel(f, F.gelu(ref_pre, approximate="tanh")) < 1e-2
    # residual accumulate: out += x @ w
    res = _rand(M, N)
    out = res.clone()
    gemm.matmul(x, w, out=out, epi="resadd")
    assert _rel(out, res.float() + x.float() @ w.float()) < 1e-2
    # dgelu + bias-gradient column sums: d = (dy @ w2^T) * gelu'(pre)
    dy = _rand(M, K)
    w2 = _rand(N, K, scale=0.1)        # logical b = w2^T [K, N] from a [N, K] tensor
    colsum = torch.zeros(N, device=DEV)
    d = gemm.matmul(dy, w2.t(), epi="dgelu", aux=pre, colsum=colsum)
    u = pre.float().requires_grad_(True)
    (gr,) = torch.autograd.grad(F.gelu(u, approximate="tanh"), u, dy.float() @ w2.float().t())
    assert _rel(d, gr) < 2e-2
    assert _rel(colsum, gr.sum(0)) < 2e-2


@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("M,N,K", [(512, 256, 128), (776, 1032, 320)])
def test_pingpong_variant_layouts(ta, tb, M, N, K):
    """variant 20 on all four operand storage forms (transposed units read with ds_read_b64_tr_b16),
    ragged M / N, plus an fp32 split-K weight-gradient accumulation (TA = TB = 1, slabs)."""
    from trustworthy_dl.ops import gemm
    a = _view(_rand(M, K), ta)
    b = _view(_rand(K, N, scale=0.1), tb)
    old = gemm.VARIANT
    gemm.VARIANT = 20
    try:
        out = gemm.matmul(a, b)
        assert _rel(out, a.float() @ b.float()) < 1e-2, (ta, tb, M, N, K)
        if ta and tb:
            acc = torch.ones(M, N, device=DEV)
            gemm.matmul_f32_acc(acc, a, b, split=2, mode="slab")
            assert _rel(acc, a.float() @ b.float() + 1.0) < 1e-4
    finally:
        gemm.VARIANT = old


@pytest.mark.parametrize("M,N,K", [(1000, 200, 128), (520, 1032, 1024), (4096, 512, 192)])
def test_pingpong_variant_epilogues(M, N, K):
    """tdl_gemm variant 20 (staggered two-group ping-pong schedule, NT operands) against fp32 torch,
    ragged M / N, the shortest K it takes (two K steps) and every epilogue it shares."""
    from trustworthy_dl.ops import gemm
    x = _rand(M, K)
    wt = _rand(N, K, scale=0.1)        # [N, K] storage: NT (forward with the W^T copy / dgrad)
    bias = _rand(N, scale=0.5)
    ref = x.float() @ wt.float().t()
    old = gemm.VARIANT
    gemm.VARIANT = 20
    try:
        y = gemm.matmul(x, wt.t(), bias=bias)
        assert _rel(y, ref + bias.float()) < 1e-2
        pre = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        f = gemm.matmul(x, wt.t(), bias=bias, epi="gelu", aux=pre)
        assert _rel(pre, ref + bias.float()) < 1e-2
        assert _rel(f, F.gelu(ref + bias.float(), approximate="tanh")) < 1e-2
        res = _rand(M, N)
        out = res.clone()
        gemm.matmul(x, wt.t(), out=out, epi="resadd")
        assert _rel(out, res.float() + ref) < 1e-2
        acc = torch.ones(M, N, device=DEV)
        gemm._launch(x, wt.t(), acc, N, "f32acc")
        assert _rel(acc, ref + 1.0) < 1e-4
    finally:
        gemm.VARIANT = old


@pytest.mark.parametrize("mode,split", [("slab", None), ("atomic", 4), ("slab", 1), ("slab", 3)])
def test_wgrad_f32(mode, split):
    from trustworthy_dl.ops import gemm
    Mt, K, N = 4096, 256, 512          # tokens, in, out
    x = _rand(Mt, K)
    dy = _rand(Mt, N)
    acc = torch.randn(K, N, device=DEV)
    base = acc.clone()
    gemm.matmul_f32_acc(acc, x.t(), dy, split=split, mode=mode)
    ref = base + x.float().t() @ dy.float()
    assert _rel(acc - base, ref - base) < 2e-3


def test_production_shape_fwd_dgrad():
    from trustworthy_dl.ops import gemm
    M, K, N = 8192, 1024, 3072
    x = _rand(M, K)
    w = _rand(K, N, scale=0.05)
    assert _rel(gemm.matmul(x, w), x.float() @ w.float()) < 1e-2
    dy = _rand(M, N)
    assert _rel(gemm.matmul(dy, w.t()), dy.float() @ w.float().t()) < 1e-2


@pytest.mark.parametrize("variant", [35, 36])
@pytest.mark.parametrize("M,N,K", [(8200, 8200, 256), (33000, 1032, 512), (4096, 2048, 1024)])
def test_persistent_pingpong_epilogues(M, N, K, variant):
    """tdl_gemm variant 35 (persistent ping-pong: > 1 tile per workgroup, the next tile's first K
    steps staged during the current tile's last, stores drained behind the next tile's MFMAs) and
    36 (LDS-staged row-contiguous epilogues: stores, and the residual / pre-activation loads) against fp32 torch on ragged M / N,
    every epilogue the GPT-2 block uses (bias, bias+GELU with the pre-activation, residual add,
    dGELU with bias-gradient column sums, fp32 accumulate)."""
    from trustworthy_dl.ops import gemm
    x = _rand(M, K)
    wt = _rand(N, K, scale=0.1)
    bias = _rand(N, scale=0.5)
    ref = x.float() @ wt.float().t()
    old = gemm.VARIANT
    gemm.VARIANT = variant
    try:
        y = gemm.matmul(x, wt.t(), bias=bias)
        assert _rel(y, ref + bias.float()) < 1e-2
        pre = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
        f = gemm.matmul(x, wt.t(), bias=bias, epi="gelu", aux=pre)
        assert _rel(pre, ref + bias.float()) < 1e-2
        assert _rel(f, F.gelu(ref + bias.float(), approximate="tanh")) < 1e-2
        res = _rand(M, N)
        out = res.clone()
        gemm.matmul(x, wt.t(), out=out, epi="resadd")
        assert _rel(out, res.float() + ref) < 1e-2
        colsum = torch.zeros(N, device=DEV)
        dy = _rand(M, K)
        d = gemm.matmul(dy, wt.t(), epi="dgelu", aux=pre, colsum=colsum)
        u = pre.float().requires_grad_(True)
        (gr,) = torch.autograd.grad(F.gelu(u, approximate="tanh"), u, dy.float() @ wt.float().t())
        assert _rel(d, gr) < 2e-2
        assert _rel(colsum, gr.sum(0)) < 2e-2
        acc = torch.ones(M, N, device=DEV)
        gemm._launch(x, wt.t(), acc, N, "f32acc")
        assert _rel(acc, ref + 1.0) < 1e-4
    finally:
        gemm.VARIANT = old
