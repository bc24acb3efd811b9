"""csrc/audit.hip against the CPU reference of security/grad_audit.py: the exact word hash must give
the same 64 bits on the GPU as on the host (the commitments of a GPU stage are checked against
recomputations that may run elsewhere), the snapshot copy must be bit-exact, and the keyed sketch
must match an fp64 host sketch with the same signs."""
import pytest
import torch

from trustworthy_dl.security import grad_audit as ga

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("n,masked", [(1, []), (1000, [(10, 20)]), (3_000_017, [(5, 700_000), (2_000_000, 2_000_001)])])
def test_word_hash_matches_host_and_snapshots(n, masked):
    from trustworthy_dl.ops import _lib
    assert _lib.lib() is not None
    torch.manual_seed(0)
    x = torch.randn(n) * 3
    x[n // 2] = float("nan")
    segs = ga._segments(n, masked)
    seed = 0xDEADBEEF
    h_cpu = int(ga.word_hash(x, segs, seed))
    xg = x.to(DEV)
    snap = torch.full((n,), 7.0, device=DEV)
    h_gpu = ga.word_hash(xg, segs, seed, snapshot=snap)
    assert int(h_gpu) == h_cpu
    keep = torch.zeros(n, dtype=torch.bool)
    for lo, hi in segs:
        keep[lo:hi] = True
    s = snap.cpu()
    assert torch.equal(s[keep].view(torch.int32), x[keep].view(torch.int32))   # bit-exact copy (NaN too)
    assert torch.all(s[~keep] == 7.0)
    # one flipped bit anywhere in a covered segment changes the hash
    y = xg.clone()
    j = segs[-1][0]
    y.view(torch.int32)[j] ^= 1
    assert int(ga.word_hash(y, segs, seed)) != h_cpu
    assert int(ga.fold_hash64(h_gpu)[0]) == int(ga.fold_hash64(torch.tensor([h_cpu]))[0])


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
