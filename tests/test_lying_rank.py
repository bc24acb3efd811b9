"""Ranks that lie in the audit protocol.

The attacker is the rank's code — a ``PipelineEngine`` subclass (attacks/lying_rank.py) — not a hook
inside an honest engine: it commits, sketches, opens and ships whatever it wants.  Against the r5
protocol all three evaded every check (scripts/lying_rank_before.py, profiles/r6_lying_rank_before.jsonl);
here each is caught by checks the auditor computes on data it hashes itself: a BLAKE2s Merkle
commitment (oracle: Python's hashlib.blake2s), keyed sketches revealed after the commitments,
openings revealed after the sketches, and a live optimizer mirror of the audited stage.
CPU: local mode (one process) and gloo ranks; tiny GPT-2 with a 1k vocabulary."""
import json
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from trustworthy_dl.security import grad_audit as ga


# ---------------------------------------------------------------------------------------------- hash
@pytest.mark.parametrize("n,segs,batch", [(1, [(0, 1)], 1), (256, [(0, 256)], 2), (257, [(0, 257)], 1),
                                          (9000, [(0, 8192), (8193, 9000)], 3), (70000, [(5, 70000)], 1),
                                          (40, [], 2)])
def test_host_merkle_matches_hashlib(n, segs, batch):
    """The C++ host tree (csrc/runtime/merkle.cpp) == hashlib.blake2s with the same node parameters."""
    x = torch.randn(n * batch)
    assert torch.equal(ga.merkle_roots(x, segs, batch=batch, stride=n),
                       ga.merkle_roots_hashlib(x, segs, batch=batch, stride=n))


def _r5_word_hash(w, seed):
    """r5's additive commitment: sum_j mix32(w_j ^ mix32(j ^ seed)) mod 2^64 (python ints)."""
    M = 0xFFFFFFFF

    def mix(x):
        x ^= x >> 16
        x = (x * 0x7feb352d) & M
        x ^= x >> 15
        x = (x * 0x6c8e9cf5) & M
        return x ^ (x >> 16)
    return sum(mix((int(v) & M) ^ mix((j & M) ^ seed)) for j, v in enumerate(w)) % (1 << 64)


def test_r5_hash_second_preimage_is_not_a_merkle_collision():
    """The r5 hash had O(1) second preimages (mix32 is invertible); the same forged buffer moves
    the Merkle root."""
    M = 0xFFFFFFFF

    def mix(x):
        x ^= x >> 16
        x = (x * 0x7feb352d) & M
        x ^= x >> 15
        x = (x * 0x6c8e9cf5) & M
        return x ^ (x >> 16)

    def unmix(y):
        y ^= y >> 16
        y = (y * pow(0x6c8e9cf5, -1, 1 << 32)) & M
        y ^= (y >> 15) ^ (y >> 30)
        y = (y * pow(0x7feb352d, -1, 1 << 32)) & M
        return y ^ (y >> 16)
    seed = 12345
    g = torch.randn(64)
    w = g.view(torch.int32).clone()
    h = _r5_word_hash(w.tolist(), seed)
    t = w.clone()
    t[3] ^= 0x80000000                                      # tamper word 3 (a sign flip)
    p = [mix((j & M) ^ seed) for j in range(64)]
    # fix one other word j so the sum is unchanged: v_j' = v_j - (v3' - v3), for a j with no wrap
    d = mix((int(t[3]) & M) ^ p[3]) - mix((int(w[3]) & M) ^ p[3])
    j = next(j for j in range(4, 64) if 0 <= mix((int(w[j]) & M) ^ p[j]) - d <= M)
    bits = unmix(mix((int(w[j]) & M) ^ p[j]) - d) ^ p[j]
    t[j] = bits - (1 << 32) if bits >= 1 << 31 else bits
    assert _r5_word_hash(t.tolist(), seed) == h              # r5: same commitment, different gradient
    assert not torch.equal(t, w)
    assert not torch.equal(ga.merkle_root(t.view(torch.float32)), ga.merkle_root(w.view(torch.float32)))


def test_keyed_sketch_batched_is_rowwise():
    n, B = 3000, 3
    a = torch.randn(B * n)
    segs = [(0, 1000), (1500, 3000)]
    key = 0x5EED_1234_ABCD
    got = ga.keyed_sketch(a, segs, key, batch=B, stride=n)
    for y in range(B):
        assert torch.allclose(got[y], ga.keyed_sketch(a[y * n:(y + 1) * n], segs, key), atol=1e-4)


# ---------------------------------------------------------------------------------------------- engines
def _batches(n, seed=0, bs=8):
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(n):
        ids = torch.randint(0, 1000, (bs, 33), generator=g)
        out.append({"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()})
    return out


def _make(nodes, kind=None, target=1, start=3, micro=4, k=4, seed=0):
    from trustworthy_dl.attacks.lying_rank import make_lying_engine
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    cls = PipelineEngine
    if kind is not None:
        cls = make_lying_engine(PipelineEngine, kind, target=target, start=start, seed=seed)
    m = get_model("gpt2-tiny", seq_len=32, seed=1, vocab_size=1024)
    return cls(m, EngineConfig(num_nodes=nodes, micro_batches=micro, device="cpu", seq_len=32, monitor_seed=seed,
                               reassign=False, audit_micro_k=k, audit_targeted=False))


def _blamed(eng):
    return sorted({(a["step"], a["node_id"], a["attack_type"]) for a in eng.attack_history})


@pytest.mark.parametrize("kind", ["lie_applied", "lie_answer", "hash_forge"])
def test_local_lying_rank_caught(kind):
    """Local mode, every micro-batch opened (k = M): each lie is caught, only the liar is blamed.
    lie_applied is caught one step later (the weights it applied leave its auditor's mirror)."""
    eng = _make(3, kind, target=1, start=3, micro=4, k=4)
    for b in _batches(6):
        eng.train_step(b)
    eng.flush()
    got = _blamed(eng)
    lied = eng.lied_steps
    assert lied == [3, 4, 5, 6]
    assert {n for _, n, _ in got} == {1}, got
    steps = {s for s, _, _ in got}
    if kind == "lie_applied":
        assert 4 in steps and all(s >= 4 for s in steps), got
        assert any(k == "model_poisoning" for _, _, k in got)
    else:
        assert set(lied) <= steps, got
        assert all(k == "gradient_poisoning" for _, _, k in got), got


def test_local_lying_sumsq_does_not_move_the_clip():
    """A stage that reports a huge gradient sum of squares would shrink every stage's update through
    the global clip scale; in mirror mode the clip uses the sums its auditor computed from the
    shipped gradient, so training is bit-identical to the clean run."""
    clean = _make(3, None, micro=2, k=2)
    liar = _make(3, "lie_sumsq", target=1, start=1, micro=2, k=2)
    for b in _batches(3):
        clean.train_step(b)
        liar.train_step(b)
    clean.flush()
    liar.flush()
    assert liar.lied_steps == [1, 2, 3]
    for n in clean.stages:
        assert torch.equal(clean.stages[n].flat.master, liar.stages[n].flat.master), n


def test_local_clean_run_no_blame_with_mirrors():
    """Clean: commitments, sums, openings, mirror weights all match for 6 steps (k = M)."""
    eng = _make(3, None, micro=4, k=4)
    for b in _batches(6):
        eng.train_step(b)
    eng.flush()
    assert _blamed(eng) == []
    s = eng.audit_summary()
    assert s["mirror_seeds"] == 3 and s["memory_bytes"] > 0       # stages 0, 1 and the loss stage
    for node, st in eng.stages.items():
        mir = [m for (v, rng), m in eng._mirrors.items() if rng == tuple(st.layer_range)]
        assert len(mir) == 1 and torch.equal(mir[0].flat.master, st.flat.master), node


@pytest.mark.parametrize("target", [0, 2])
def test_local_lying_tied_member_caught(target):
    """The tied embedding / LM-head gradient: a member applying (and committing, and shipping) a
    sign-flipped tied gradient passes its own sum check (the tied rows are the all-reduce's) and is
    caught by the cross-member tie check, computed by the two members' auditors only."""
    eng = _make(3, "lie_tied", target=target, start=3, micro=4, k=1)
    for b in _batches(6):
        eng.train_step(b)
    eng.flush()
    got = _blamed(eng)
    assert eng.lied_steps == [3, 4, 5, 6]
    assert {n for _, n, _ in got} == {target}, got
    assert set(eng.lied_steps) <= {s for s, _, _ in got}, got


def test_local_lying_tied_feed_is_skipped_not_blamed():
    """A member feeding the tied all-reduce something else than its committed contributions makes
    both members apply the same wrong sum: not attributable, so nobody is blamed and every such
    step's update is skipped — the weights never move off the last clean step's."""
    eng = _make(3, "lie_tied_feed", target=2, start=3, micro=2, k=1)
    bs = _batches(5)
    for b in bs[:2]:
        eng.train_step(b)
    eng.flush()
    before = {n: st.flat.master.clone() for n, st in eng.stages.items()}
    for b in bs[2:]:
        eng.train_step(b)
    eng.flush()
    assert eng.lied_steps == [3, 4, 5]
    assert _blamed(eng) == []
    for n, st in eng.stages.items():
        assert torch.equal(st.flat.master, before[n]), n


# ---------------------------------------------------------------------------------------------- gloo ranks
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path, kind, target, micro, k, steps, seed):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = _make(world, kind if rank == target else None, target=target, start=3, micro=micro, k=k, seed=seed)
    for b in _batches(steps, seed=seed, bs=2 * micro):
        eng.train_step(b)
    eng.flush()
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump({"blamed": _blamed(eng), "lied": getattr(eng, "lied_steps", []), "audit": eng.audit_summary()}, f)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


def _run_gloo(world, kind, target, micro, k, steps, seed=0):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "r")
        mp.spawn(_worker, args=(world, _free_port(), out, kind, target, micro, k, steps, seed), nprocs=world, join=True)
        return [json.load(open(f"{out}.{r}")) for r in range(world)]


@pytest.mark.parametrize("kind,target", [("lie_applied", 1), ("lie_answer", 1), ("hash_forge", 2),
                                         ("lie_answer", 0), ("lie_tied", 2)])
@pytest.mark.slow
def test_gloo_lying_rank_caught(kind, target):
    """3 gloo processes, the liar is a subclass in its own process (the loss stage for hash_forge,
    the first stage for one lie_answer run); every micro-batch opened: caught, every rank agrees,
    nobody else blamed."""
    res = _run_gloo(3, kind, target, micro=4, k=4, steps=7)
    assert all(r["blamed"] == res[0]["blamed"] for r in res)
    got = res[0]["blamed"]
    lied = res[target]["lied"]
    assert lied == [3, 4, 5, 6, 7]
    assert {n for _, n, _ in got} == {target}, got
    steps = {s for s, _, _ in got}
    if kind == "lie_applied":
        assert min(steps) == 4, got
    else:
        assert set(lied) <= steps, got


@pytest.mark.slow
def test_gloo_lying_rank_one_of_m():
    """k = 1 of M = 4: lie_answer is caught only when its lied micro-batch is opened (~1/4 of the
    steps) — never a clean rank; the mirrors keep every stage's weights bit-identical."""
    res = _run_gloo(3, "lie_answer", 1, micro=4, k=1, steps=14)
    assert all(r["blamed"] == res[0]["blamed"] for r in res)
    got = res[0]["blamed"]
    assert {n for _, n, _ in got} <= {1}
    assert got, "never caught in 12 lying steps at k/M = 1/4"
    a = res[2]["audit"]
    assert a["mirror_seeds"] == 1 and a["steps"] == 14


# ---------------------------------------------------------------------------------------------- healing
def _heal_worker(rank, world, port, out_path, steps):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from trustworthy_dl.attacks import AdversarialAttacker, AttackConfig
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    atk = AdversarialAttacker(AttackConfig(["model_poisoning"], target_nodes=[1], intensity=0.05, start_step=3,
                                           end_step=3))
    atk.activate_attacks()
    m = get_model("gpt2-tiny", seq_len=32, seed=1, vocab_size=1024)
    eng = PipelineEngine(m, EngineConfig(num_nodes=world, micro_batches=2, device="cpu", seq_len=32, monitor_seed=0,
                                         reassign=False, audit_micro_k=1, audit_targeted=False),
                         attacker=atk)
    for b in _batches(steps, bs=4):
        eng.train_step(b)
    eng.flush()
    st = eng.my_stage()
    rec = {"blamed": _blamed(eng), "master": ga.root_hex(ga.merkle_root(st.flat.master)),
           "heals": eng.audit_summary().get("heals", 0) if hasattr(eng, "audit_summary") else 0}
    if rank == 2:   # the auditor of stage 1: its mirror's master
        mir = [m_ for (v, rng), m_ in eng._mirrors.items() if rng == tuple(eng.plan.ranges[1])]
        rec["mirror_of_1"] = ga.root_hex(ga.merkle_root(mir[0].flat.master))
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump(rec, f)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
def test_gloo_tampered_weights_healed_from_the_auditors_mirror():
    """3 gloo ranks, stage 1's weights perturbed once (step 3, outside the optimizer), no re-shard:
    blamed from step 3 until the step-3 report is processed (REPORT_LAG steps later), when its
    auditor ships the mirror's verified optimizer state and the stage adopts it — no blame after
    that, and its master weights equal the mirror's bit for bit."""
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "h")
        mp.spawn(_heal_worker, args=(3, _free_port(), out, 9), nprocs=3, join=True)
        res = [json.load(open(f"{out}.{r}")) for r in range(3)]
    got = res[0]["blamed"]
    assert all(r["blamed"] == got for r in res)
    steps = sorted({s for s, n, _ in got})
    assert {n for _, n, _ in got} == {1} and steps and steps[0] == 3 and steps[-1] <= 5, got
    assert res[1]["master"] == res[2]["mirror_of_1"]
