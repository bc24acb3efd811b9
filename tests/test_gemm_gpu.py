"""Native MFMA GEMMs (csrc/gemm.hip: p4 = persistent 4-wave kernel, p4l = the same with the
LDS-staged epilogue, pp = staggered 8-wave ping-pong kernel, pd = persistent 4-wave kernel with
LDS-DMA staging, NT operands only) vs a plain PyTorch fp32 reference of the same op (GPU only).

Covers the four operand storage forms (k-contiguous / row-contiguous for A and B), every fused
epilogue, ragged M and N (tile clamping + store masks), split-K slabs and atomics, and every
product the engine routes to a native kernel at its production GPT-2-medium shape (64k tokens,
K up to 4096)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
KERNELS = ["p4", "p4l", "pp"]
NT_KERNELS = KERNELS + ["pd"]      # pd takes k-contiguous (NT) operands; others fall back to pp


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


@pytest.mark.parametrize("kernel", NT_KERNELS)
@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
@pytest.mark.parametrize("M,N,K", [(512, 256, 128), (776, 1032, 320), (8200, 520, 512)])
def test_layouts(kernel, ta, tb, M, N, K):
    """all four storage forms, ragged M / N, > 1 tile per persistent workgroup (8200 rows), plus an
    fp32 split-K accumulation through slabs"""
    from trustworthy_dl.ops import gemm
    a = _view(_rand(M, K), ta)
    b = _view(_rand(K, N, scale=0.1), tb)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    gemm._launch(a, b, out, N, "none", kernel=kernel)
    ref = a.float() @ b.float()
    assert _rel(out, ref) < 1e-2, (kernel, ta, tb, M, N, K)
    acc = torch.ones(M, N, device=DEV)
    gemm.matmul_f32_acc(acc, a, b, split=2, mode="slab", kernel=kernel)
    assert _rel(acc, ref + 1.0) < 1e-4


@pytest.mark.parametrize("kernel", NT_KERNELS)
@pytest.mark.parametrize("M,N,K", [(1000, 200, 128), (8200, 1032, 256), (4096, 2048, 1024)])
def test_epilogues(kernel, M, N, K):
    """every epilogue the GPT-2 block uses (bias, bias+GELU with the pre-activation, residual add,
    dGELU with bias-gradient column sums, fp32 accumulate / slabs / atomics), NT operands, ragged"""
    from trustworthy_dl.ops import gemm
    x = _rand(M, K)
    wt = _rand(N, K, scale=0.1)        # [N, K] storage: NT (forward with the W^T copy / dgrad)
    bias = _rand(N, scale=0.5)
    ref = x.float() @ wt.float().t()

    def mm(out, epi, **kw):
        gemm._launch(x, wt.t(), out, N, epi, kernel=kernel, **kw)
        return out
    y = mm(torch.empty(M, N, dtype=torch.bfloat16, device=DEV), "none", bias=bias)
    assert _rel(y, ref + bias.float()) < 1e-2
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    f = mm(torch.empty(M, N, dtype=torch.bfloat16, device=DEV), "gelu", bias=bias, aux=pre)
    assert _rel(pre, ref + bias.float()) < 1e-2
    assert _rel(f, F.gelu(ref + bias.float(), approximate="tanh")) < 1e-2
    res = _rand(M, N)
    out = mm(res.clone(), "resadd")
    assert _rel(out, res.float() + ref) < 1e-2
    colsum = torch.zeros(N, device=DEV)
    dy = _rand(M, K)
    d = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    gemm._launch(dy, wt.t(), d, N, "dgelu", aux=pre, colsum=colsum, kernel=kernel)
    u = pre.float().requires_grad_(True)
    (gr,) = torch.autograd.grad(F.gelu(u, approximate="tanh"), u, dy.float() @ wt.float().t())
    assert _rel(d, gr) < 2e-2
    assert _rel(colsum, gr.sum(0)) < 2e-2
    acc = mm(torch.ones(M, N, device=DEV), "f32acc")
    assert _rel(acc, ref + 1.0) < 1e-4
    for mode in ("slab", "atomic"):
        acc = torch.ones(M, N, device=DEV)
        gemm.matmul_f32_acc(acc, x, wt.t(), split=2, mode=mode, kernel=kernel)
        assert _rel(acc, ref + 1.0) < 1e-4, mode


@pytest.mark.parametrize("group", ["0", "8", "3"])
def test_tile_orders(group, monkeypatch):
    """every tile order (row-major, grouped by 8 tile rows, a group size that leaves a partial last
    group) covers every output tile exactly once: ragged M / N, ping-pong and persistent kernels"""
    from trustworthy_dl.ops import gemm
    monkeypatch.setenv("TDL_GEMM_GROUPM", group)
    M, N, K = 2824, 4360, 256          # 12 x 18 tiles
    x = _rand(M, K)
    wt = _rand(N, K, scale=0.1)
    ref = x.float() @ wt.float().t()
    for kn in ("pp", "p4", "p4l", "pd"):
        out = torch.full((M, N), float("nan"), dtype=torch.bfloat16, device=DEV)
        gemm._launch(x, wt.t(), out, N, "none", kernel=kn)
        assert _rel(out, ref) < 1e-2, (kn, group)


def test_dgelu_rejects_transposed_a():
    """the dGELU column sums need rows past M to read as zero, which a transposed A cannot give"""
    from trustworthy_dl.ops import gemm
    a = _view(_rand(264, 128), True)
    with pytest.raises(ValueError):
        gemm.matmul(a, _rand(128, 256), epi="dgelu", aux=torch.empty(264, 256, dtype=torch.bfloat16, device=DEV),
                    colsum=torch.zeros(256, device=DEV))


@pytest.mark.parametrize("kernel", ["p4", "pd"])
@pytest.mark.parametrize("mode,split", [("slab", None), ("atomic", 4), ("slab", 1), ("slab", 3)])
def test_wgrad_f32(mode, split, kernel):
    from trustworthy_dl.ops import gemm
    Mt, K, N = 4096, 256, 512          # tokens, in, out
    x = _rand(Mt, K)
    dy = _rand(Mt, N)
    acc = torch.randn(K, N, device=DEV)
    base = acc.clone()
    gemm.matmul_f32_acc(acc, x.t(), dy, split=split, mode=mode, kernel=kernel)
    ref = base + x.float().t() @ dy.float()
    assert _rel(acc - base, ref - base) < 2e-3


@pytest.mark.parametrize("Mt,K,N,split", [(65536, 1024, 3072, 16), (65536, 4096, 1024, 4), (4096, 1000, 264, 2),
                                          (16384, 50304, 1024, 4)])
def test_wgrad_pd_transposed_operands(Mt, K, N, split):
    """The LDS-DMA kernel on the weight-gradient layout (both operands row-contiguous, read with
    ds_read_b64_tr_b16; copies issued from asm): production shapes, ragged tiles, the LM head."""
    from trustworthy_dl.ops import gemm
    x = _rand(Mt, K)
    dy = _rand(Mt, N, scale=0.1)
    acc = torch.randn(K, N, device=DEV)
    ref = acc + x.float().t() @ dy.float()
    gemm.matmul_f32_acc(acc, x.t(), dy, split=split, kernel="pd")
    assert float((acc - ref).norm() / ref.norm()) < 1e-4
    acc2 = torch.zeros(K, N, device=DEV)   # bit-identical to a second run (deterministic split reduce)
    acc3 = torch.zeros(K, N, device=DEV)
    gemm.matmul_f32_acc(acc2, x.t(), dy, split=split, kernel="pd")
    gemm.matmul_f32_acc(acc3, x.t(), dy, split=split, kernel="pd")
    assert torch.equal(acc2, acc3)


# every product the engine routes to a native kernel, at the production shape (64k tokens)
@pytest.mark.parametrize("name,tokens,cin,cout", [("qkv", 65536, 1024, 3072), ("o", 65536, 1024, 1024),
                                                  ("fc", 65536, 1024, 4096), ("proj", 65536, 4096, 1024)])
def test_production_wgrad(name, tokens, cin, cout):
    """dW += x^T dy (fp32 main_grad) for the four projections of a GPT-2-medium block"""
    from trustworthy_dl.ops.layers import wgrad_acc
    x = _rand(tokens, cin)
    dy = _rand(tokens, cout, scale=0.1)
    acc = torch.randn(cin, cout, device=DEV)
    ref = acc + x.float().t() @ dy.float()
    wgrad_acc(acc, x.t(), dy)
    assert float((acc - ref).norm() / ref.norm()) < 1e-4, name


def test_production_lm_head_wgrad():
    """tied LM head dW += dlogits^T x at V = 50304 (padded), 16k tokens, K = tokens"""
    from trustworthy_dl.ops.layers import wgrad_acc
    dl = _rand(16384, 50304, scale=0.01)
    x = _rand(16384, 1024)
    acc = torch.zeros(50304, 1024, device=DEV)
    wgrad_acc(acc, dl.t(), x)
    ref = dl.float().t() @ x.float()
    assert float((acc - ref).norm() / ref.norm()) < 1e-4


def test_production_fused_mlp():
    """the MLP GEMMs the block fuses on the ping-pong kernel: fc forward (bias + GELU, pre-activation
    stored, K = 1024) and proj dgrad (dGELU + bias-gradient column sums, K = 1024), and the
    K = 4096 proj forward with the residual-add epilogue, at 64k tokens"""
    from trustworthy_dl.ops import gemm
    M = 65536
    h = _rand(M, 1024)
    wfc_t = _rand(4096, 1024, scale=0.05)
    bfc = _rand(4096, scale=0.5)
    pre = torch.empty(M, 4096, dtype=torch.bfloat16, device=DEV)
    f = gemm.matmul(h, wfc_t.t(), bias=bfc, epi="gelu", aux=pre)
    ref = h.float() @ wfc_t.float().t() + bfc.float()
    assert _rel(pre, ref) < 1e-2
    assert _rel(f, F.gelu(ref, approximate="tanh")) < 1e-2
    del ref
    dy = _rand(M, 1024)
    wp = _rand(4096, 1024, scale=0.05)                 # W_proj [in 4096, out 1024]
    colsum = torch.zeros(4096, device=DEV)
    d = gemm.matmul(dy, wp.t(), epi="dgelu", aux=pre, colsum=colsum)
    u = pre.float().requires_grad_(True)
    (gr,) = torch.autograd.grad(F.gelu(u, approximate="tanh"), u, dy.float() @ wp.float().t())
    assert _rel(d, gr) < 2e-2
    assert _rel(colsum, gr.sum(0)) < 2e-2
    del u, gr
    y = _rand(M, 1024)
    y0 = y.float()
    gemm.matmul(f, wp, out=y, epi="resadd")
    assert _rel(y, y0 + f.float() @ wp.float()) < 1e-2


@pytest.mark.parametrize("Mt,K,N1,K2,N2", [(65536, 1024, 3072, 1024, 1024), (16384, 1024, 3072, 1024, 1024),
                                            (65536, 1024, 4096, 4096, 1024), (4096, 264, 520, 136, 200)])
def test_wgrad_grouped_pair(Mt, K, N1, K2, N2):
    """qkv + o (and fc + proj: different input widths) weight gradients from ONE grouped launch
    (tdl_gemm_wgrad_grouped: one output tile x slice per workgroup, product chosen per workgroup) vs
    fp32, ragged tiles included; deterministic; a pair whose items do not fit one round on the CUs
    is declined (caller runs them separately)."""
    from trustworthy_dl.ops import gemm
    x1, x2 = _rand(Mt, K), _rand(Mt, K2)
    d1, d2 = _rand(Mt, N1, scale=0.1), _rand(Mt, N2, scale=0.1)
    acc1, acc2 = torch.randn(K, N1, device=DEV), torch.randn(K2, N2, device=DEV)
    ref1 = acc1 + x1.float().t() @ d1.float()
    ref2 = acc2 + x2.float().t() @ d2.float()
    assert gemm.matmul_f32_acc_grouped(acc1, x1.t(), d1, acc2, x2.t(), d2)
    assert float((acc1 - ref1).norm() / ref1.norm()) < 1e-4
    assert float((acc2 - ref2).norm() / ref2.norm()) < 1e-4
    r = []
    for _ in range(2):
        a1, a2 = torch.zeros(K, N1, device=DEV), torch.zeros(K2, N2, device=DEV)
        assert gemm.matmul_f32_acc_grouped(a1, x1.t(), d1, a2, x2.t(), d2)
        r.append((a1, a2))
    assert torch.equal(r[0][0], r[1][0]) and torch.equal(r[0][1], r[1][1])
    # the slabs path of the separate launches gives the same sums up to fp32 reassociation
    s1 = torch.zeros(K, N1, device=DEV)
    gemm.matmul_f32_acc(s1, x1.t(), d1, kernel="pd")
    assert float((s1 - r[0][0]).norm() / s1.norm()) < 1e-5


def test_wgrad_grouped_declines_oversized():
    from trustworthy_dl.ops import gemm
    Mt, K = 1024, 8192                                   # 32 x 16 tiles: more than one round
    x = _rand(Mt, K)
    d = _rand(Mt, 4096)
    acc = torch.zeros(K, 4096, device=DEV)
    assert not gemm.matmul_f32_acc_grouped(acc, x.t(), d, acc.clone(), x.t(), d)
    assert float(acc.abs().max()) == 0.0
