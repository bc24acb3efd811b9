"""Commit-then-reveal gradient audit against an ADAPTIVE adversary.

r4's gradient commitments were sketches under PUBLIC sign patterns over a public 1/16 sample of
the gradient (security/grad_audit.GradSketch): an adversary that knows the job seed, the step and
the stage's layer range tampers only the coordinates the sketch does not read, and both checks —
applied-vs-committed and the audited micro-batch's recomputed contribution — pass.  The binding
checks are now BLAKE2s Merkle commitments of every micro-batch's contribution and of the applied
gradient (every coordinate), keyed full-coverage sketches under a key the auditor reveals only after
it received the commitments, and a live optimizer mirror (csrc/audit.hip, parallel/commitments.py).
CPU, local mode; tiny GPT-2."""
import pytest
import torch

from trustworthy_dl.security import grad_audit as ga


def _engine(nodes, targets=(1,), start=4, micro=4, atk_kw=None, **cfg):
    from trustworthy_dl.attacks.adversarial_attacks import AdversarialAttacker, AttackConfig
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    att = AdversarialAttacker(AttackConfig(attack_types=["gradient_poisoning"], target_nodes=list(targets),
                                           intensity=0.5, start_step=start, probability=1.0, seed=3,
                                           adaptive=True, gradient_mode="sign_flip", **(atk_kw or {})))
    att.activate_attacks()
    cfg.setdefault("reassign", False)
    cfg.setdefault("audit_targeted", False)
    m = get_model("gpt2-tiny", seq_len=32, seed=1, vocab_size=1024)
    return PipelineEngine(m, EngineConfig(num_nodes=nodes, micro_batches=micro, device="cpu", seq_len=32,
                                          monitor_seed=0, **cfg), attacker=att), att


def _batches(n, seed=0, bs=8):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        ids = torch.randint(0, 1000, (bs, 33), generator=g)
        out.append({"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()})
    return out


def _blamed(eng):
    return sorted({(a["step"], a["node_id"], a["attack_type"]) for a in eng.attack_history})


def test_adaptive_tamper_is_invisible_to_the_public_sketch():
    """The attack the old protocol could not see: a sign flip of every coordinate the public
    sketch does not sample leaves that sketch bit-identical, while the exact hash and the keyed
    sketch move by the size of the tamper."""
    n = 1 << 16
    g = torch.randn(n)
    sk = ga.GradSketch(n, "cpu", seed=7)
    off = sk.offset(0, 5)
    delta = -2.0 * g
    delta[: sk.nblk * sk.block].view(sk.nblk, sk.block)[:, off:off + sk.win] = 0.0
    t = g + delta
    assert torch.equal(sk(g, off), sk(t, off))                      # r4's commitment: no difference
    segs = ga._segments(n)
    assert not torch.equal(ga.merkle_root(g, segs), ga.merkle_root(t, segs))
    key = 0x1234_5678_9ABC
    a, b = ga.keyed_sketch(g, segs, key), ga.keyed_sketch(t, segs, key)
    assert float((a - b).abs().max()) > 0.5 * float(delta.norm())   # ~ ||delta|| per sign vector


def test_keyed_sketch_linear_and_masked():
    """Linear (the answer for a contribution is the sketch of a snapshot difference), blind to the
    masked (tied-weight) range, and a fresh key gives fresh signs."""
    n = 5000
    a, b = torch.randn(n), torch.randn(n)
    segs = ga._segments(n, [(1000, 2000)])
    k = 987654321
    s_ab = ga.keyed_sketch(a, segs, k, b=b)
    assert torch.allclose(s_ab, ga.keyed_sketch(a, segs, k) - ga.keyed_sketch(b, segs, k), atol=1e-3)
    a2 = a.clone()
    a2[1500] += 100.0
    assert torch.equal(ga.keyed_sketch(a2, segs, k), ga.keyed_sketch(a, segs, k))
    assert torch.equal(ga.merkle_root(a2, segs), ga.merkle_root(a, segs))
    assert not torch.allclose(ga.keyed_sketch(a, segs, k), ga.keyed_sketch(a, segs, k + 1))


def test_local_adaptive_post_backward_caught_every_step():
    """Adaptive tamper between backward and optimizer: the applied gradient's keyed sketch is no
    longer the sum of the committed contributions' on every tampered step; only the target is blamed."""
    eng, att = _engine(3, targets=(1,), start=4, micro=2)
    for b in _batches(8):
        eng.train_step(b)
    eng.flush()
    got = _blamed(eng)
    tampered = sorted({r["step"] for r in att.injections})
    assert tampered == list(range(4, 9))
    assert {n for _, n, _ in got} == {1}, got
    assert {s for s, _, _ in got} == set(tampered)


@pytest.mark.parametrize("k", [pytest.param(1, marks=pytest.mark.slow), 4])
def test_local_adaptive_one_of_m_caught_by_keyed_recompute(k):
    """Adaptive tamper of ONE micro-batch's contribution inside the backward (consistent with the
    commitments): only the keyed recompute of an audited micro-batch sees it.  With k = M audited
    micro-batches every tampered step is caught; with k = 1 the expected wait is M / k steps.
    Clean stages are never blamed."""
    M = 4
    eng, att = _engine(3, targets=(1,), start=3, micro=M, atk_kw={"micro_batches": 1}, audit_micro_k=k)
    steps = 14 if k == 1 else 6
    for b in _batches(steps):
        eng.train_step(b)
    eng.flush()
    got = _blamed(eng)
    tampered = sorted({r["step"] for r in att.injections})
    assert tampered, "attack never fired"
    assert got, "adaptive one-of-M tamper never caught"
    assert {n for _, n, _ in got} == {1}, got
    assert all(kind == "gradient_poisoning" for _, _, kind in got)
    if k == M:
        assert {s for s, _, _ in got} == set(tampered)


@pytest.mark.slow
def test_local_clean_run_no_false_keyed_flags():
    """No attack: the keyed recompute and the exact applied hash never flag a clean stage, k = M."""
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    m = get_model("gpt2-tiny", seq_len=32, seed=1, vocab_size=1024)
    eng = PipelineEngine(m, EngineConfig(num_nodes=3, micro_batches=4, device="cpu", seq_len=32, monitor_seed=0,
                                         reassign=False, audit_micro_k=4))
    for b in _batches(6):
        eng.train_step(b)
    eng.flush()
    assert _blamed(eng) == []
