"""csrc/audit.hip against the host references of security/grad_audit.py: the BLAKE2s Merkle roots
must be bit-identical on the GPU, in the C++ host runtime and in Python's hashlib (commitments made
on one GPU are checked by an auditor on another, and CPU ranks use the host path); the keyed sketch
must match an fp64 host sketch with the same signs and be deterministic (the auditor compares the
auditee's value bit for bit); the contribution snapshot is an exact fp32 subtraction.  Then the whole
protocol on the GPU engine: a clean local-mode run raises no flag (the recompute of an opened
contribution on the mirror matches the committed one on the native kernels) and a lying stage is
caught."""
import pytest
import torch

from trustworthy_dl.security import grad_audit as ga

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("n,segs,batch", [(1, [(0, 1)], 1), (1000, [(3, 10), (20, 1000)], 2),
                                          (256 * 33 + 5, [(0, 256 * 33 + 5)], 3),
                                          (3_000_017, [(5, 700_000), (700_001, 3_000_017)], 1),
                                          (512, [], 1)])
def test_merkle_gpu_matches_host_and_hashlib(n, segs, batch):
    from trustworthy_dl.ops import _lib
    assert _lib.lib() is not None
    torch.manual_seed(0)
    x = torch.randn(n * batch) * 3
    x[n // 2] = float("nan")
    host = ga.merkle_roots(x, segs, batch=batch, stride=n)
    gpu = ga.merkle_roots(x.to(DEV), segs, batch=batch, stride=n)
    assert gpu.is_cuda
    assert torch.equal(gpu.cpu(), host)
    if n * batch <= 100_000:
        assert torch.equal(host, ga.merkle_roots_hashlib(x, segs, batch=batch, stride=n))
    if segs:   # one flipped bit anywhere in a covered segment changes the root
        y = x.to(DEV).clone()
        y.view(torch.int32)[segs[-1][1] - 1] ^= 1
        assert not torch.equal(ga.merkle_roots(y, segs, batch=batch, stride=n)[0].cpu(), host[0])


@pytest.mark.parametrize("n", [4096, 2_500_003])
def test_keyed_sketch_matches_host(n):
    torch.manual_seed(1)
    a, b = torch.randn(n), torch.randn(n)
    segs = ga._segments(n, [(100, 900)])
    key = 0x0123_4567_89AB_CDEF
    k0, k1 = ga.key_words(key)
    j = torch.arange(n, dtype=torch.int64) & ga.M32
    h = ga._mix32(ga._mix32(j ^ k0) ^ k1)
    keep = torch.zeros(n, dtype=torch.bool)
    for lo, hi in segs:
        keep[lo:hi] = True
    v = (a.double() - b.double()) * keep.double()
    ref = torch.stack([((1.0 - 2.0 * ((h >> (28 + k)) & 1).double()) * v).sum() for k in range(ga.K_KEYED)])
    got = ga.keyed_sketch(a.to(DEV), segs, key, b=b.to(DEV)).double().cpu()
    scale = float(v.norm())
    assert float((got - ref).abs().max()) < 1e-5 * scale
    got2 = ga.keyed_sketch(a.to(DEV), segs, key, b=b.to(DEV)).cpu()
    assert torch.equal(got2.double(), got)   # fixed reduction order: deterministic
    # batched rows == single sketches, bit for bit
    B = 3
    ab = torch.randn(B * n, device=DEV)
    rows = ga.keyed_sketch(ab, segs, key, batch=B, stride=n)
    for y in range(B):
        assert torch.equal(rows[y], ga.keyed_sketch(ab[y * n:(y + 1) * n], segs, key))


def test_contrib_snap_exact():
    torch.manual_seed(2)
    n = 1_000_003
    g, prev = torch.randn(n, device=DEV), torch.randn(n, device=DEV)
    c = torch.empty(n, device=DEV)
    want = g - prev
    ga.contrib_snap(g, prev, c)
    assert torch.equal(c, want) and torch.equal(prev, g)


def _engine(kind=None, k=4):
    from trustworthy_dl.attacks.lying_rank import make_lying_engine
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    cls = PipelineEngine if kind is None else make_lying_engine(PipelineEngine, kind, target=1, start=3)
    m = get_model("gpt2-tiny", seq_len=128, seed=1)
    return cls(m, EngineConfig(num_nodes=3, micro_batches=4, device="cuda:0", seq_len=128, monitor_seed=0,
                               reassign=False, audit_micro_k=k, audit_targeted=False))


def _batches(n, bs=8, T=128):
    g = torch.Generator().manual_seed(0)
    out = []
    for _ in range(n):
        ids = torch.randint(0, 50257, (bs, T + 1), generator=g)
        out.append({"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()})
    return out


@pytest.mark.parametrize("kind", [None, "lie_answer", "lie_applied"])
def test_gpu_local_protocol(kind):
    """bf16 GPU engine, 3 stages on one GPU, every micro-batch opened: clean -> no flag and every
    mirror bit-identical to its stage; a lying stage -> blamed, nobody else."""
    eng = _engine(kind)
    for b in _batches(6):
        eng.train_step(b)
    eng.flush()
    torch.cuda.synchronize()
    blamed = sorted({(a["step"], a["node_id"]) for a in eng.attack_history})
    if kind is None:
        assert blamed == [], (blamed, [a.get("audit_kind") for a in eng.attack_history])
        for st in eng.stages.values():
            mir = [m for (v, rng), m in eng._mirrors.items() if rng == tuple(st.layer_range)]
            assert len(mir) == 1 and torch.equal(mir[0].flat.master, st.flat.master)
    else:
        assert blamed and {n for _, n in blamed} == {1}, blamed


def test_seg_rel_err_matches_torch():
    torch.manual_seed(3)
    n = 2_000_003
    a, b = torch.randn(n, device=DEV), torch.randn(n, device=DEV)
    segs = [(0, 1000), (5000, n)]
    got = float(ga.seg_rel_err(a, b, segs))
    keep = torch.zeros(n, dtype=torch.bool, device=DEV)
    for lo, hi in segs:
        keep[lo:hi] = True
    want = float((a - b).abs()[keep].max() / b.abs()[keep].max())
    assert got == pytest.approx(want, rel=1e-6)
    a[7000] = float("nan")
    assert float(ga.seg_rel_err(a, b, segs)) >= 1e29          # NaN reads as the largest error
    assert float(ga.seg_sumsq(b, segs)) == pytest.approx(float(b[keep].double().square().sum()), rel=1e-4)
