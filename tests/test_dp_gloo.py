"""Data parallelism over pipeline replicas (CPU/gloo): world = stages x replicas.

* pp2 x dp2 must train exactly like the single-process 2-stage engine on the same global batch
  (replica gradients are averaged; the global-norm clip sees the aggregated gradient);
* a replica whose weights are tampered with is caught by the cross-replica parameter audit,
  marked compromised and re-synchronised from the majority (dp3)."""
import json
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches(n, bs):
    g = torch.Generator().manual_seed(11)
    out = []
    for _ in range(n):
        ids = torch.randint(0, 1000, (bs, 33), generator=g)
        out.append({"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()})
    return out


def _engine(nodes, micro, dp=1, audit=0):
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.flat import AdamWConfig
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    from trustworthy_dl.utils.metrics import MetricsCollector
    m = get_model("gpt2-tiny", seed=3, seq_len=32, vocab_size=1024)
    cfg = EngineConfig(num_nodes=nodes, micro_batches=micro, device="cpu", seq_len=32, data_parallel=dp,
                       param_audit_interval=audit, reassign=False,
                       adamw=AdamWConfig(lr=1e-2, eps=1.0, max_grad_norm=1.0))
    return PipelineEngine(m, cfg, metrics=MetricsCollector())


def _worker(rank, world, port, dp, steps, tamper_step, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = _engine(world // dp, 2, dp=dp, audit=2 if tamper_step else 0)
    for i, b in enumerate(_batches(steps, 4 * dp)):
        eng.train_step(b)
        if tamper_step and i + 1 == tamper_step and rank == 1:
            st = eng.my_stage()
            with torch.no_grad():
                st.flat.master.add_(torch.randn_like(st.flat.master) * 1e-2)
                st.flat.data.copy_(st.flat.master)
    eng.flush()
    sd = eng.stage_state_dicts()
    res = {"losses": [m["loss"] for m in eng.metrics.batch_metrics],
           "weights": {n: float(t.double().sum()) for s_ in sd.values() for n, t in s_.items()},
           "audits": eng.dp_audits, "trust": [eng.trust.get_trust_score(i) for i in range(world)],
           "status": [eng.trust.get_node_status(i).value for i in range(world)]}
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


def _run(world, dp, steps, tamper_step=0):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "res")
        mp.spawn(_worker, args=(world, _free_port(), dp, steps, tamper_step, out), nprocs=world, join=True)
        return [json.load(open(f"{out}.{r}")) for r in range(world)]


def test_pp2_dp2_matches_single_process():
    steps = 4
    res = _run(4, 2, steps)  # global batch 8 = 2 replicas x 4
    torch.set_num_threads(4)
    local = _engine(2, 2)
    for b in _batches(steps, 8):
        local.train_step(b)
    local.flush()
    ref = [m["loss"] for m in local.metrics.batch_metrics]
    for r in range(4):
        assert res[r]["losses"] == pytest.approx(ref, rel=2e-3)
    lw = local.stage_state_dicts()
    for r in range(4):
        stage = r % 2
        for n, v in res[r]["weights"].items():
            assert v == pytest.approx(float(lw[stage][n].double().sum()), rel=1e-4, abs=1e-5), (r, n)


def test_dp3_param_audit_catches_and_resyncs_tampered_replica():
    res = _run(3, 3, steps=5, tamper_step=3)
    for r in range(3):
        audits = res[r]["audits"]
        assert audits and audits[0]["divergent_nodes"] == [1] and audits[0]["step"] == 4
        assert res[r]["status"][1] == "compromised"
    # after the re-sync every replica holds the same weights again
    w0 = res[0]["weights"]
    for r in (1, 2):
        for n, v in res[r]["weights"].items():
            assert v == pytest.approx(w0[n], rel=1e-6, abs=1e-7), (r, n)


class _ScaleAttacker:
    """Scales node 1's gradient by 50 every step (gradient poisoning of one replica)."""

    def on_gradients(self, node, grad, step):
        if node == 1:
            grad.mul_(50.0)
            return True
        return False


class _NaNAttacker:
    """Writes NaN / Inf into node 1's gradient every step (a replica producing non-finite values)."""

    def on_gradients(self, node, grad, step):
        if node == 1:
            grad[:64] = float("nan")
            grad[64:128] = float("inf")
            return True
        return False


class _SignFlipAttacker:
    """Negates node 1's gradient every step (its norm and statistics stay normal)."""

    def on_gradients(self, node, grad, step):
        if node == 1:
            grad.neg_()
            return True
        return False


def _attack_worker(rank, world, port, out_path, kind="scale"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = _engine(1, 2, dp=3)
    eng.attacker = {"scale": _ScaleAttacker, "nan": _NaNAttacker, "sign_flip": _SignFlipAttacker}[kind]()
    excluded = []
    if kind == "sign_flip":   # replicas must share a learning signal for a direction test: Markov tokens
        from trustworthy_dl.utils.data_loader import MarkovLanguageModeling
        batches = list(MarkovLanguageModeling(12, 32, 64, num_batches=3, seed=2))
    else:
        batches = _batches(3, 12)
    for b in batches:
        eng.train_step(b)
        excluded.append([int(v) for v in eng._dp_excluded.tolist()])
    eng.flush()
    sd = eng.stage_state_dicts()
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump({"excluded": excluded,
                   "weights": {n: float(t.double().sum()) for s_ in sd.values() for n, t in s_.items()}}, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["scale", "nan", "sign_flip"])
def test_dp3_robust_aggregation_excludes_poisoned_replica(kind):
    """x50 gradients, NaN/Inf gradients or a sign-flipped gradient (caught only by the cross-replica
    direction check) on one replica: it is left out of the mean and every replica (the poisoned
    one included) ends with the same finite weights."""
    import math
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "res")
        mp.spawn(_attack_worker, args=(3, _free_port(), out, kind), nprocs=3, join=True)
        res = [json.load(open(f"{out}.{r}")) for r in range(3)]
    for r in range(3):
        assert res[r]["excluded"] == [[0, 1, 0]] * 3
        assert all(math.isfinite(v) for v in res[r]["weights"].values())
    for r in (1, 2):
        for n, v in res[r]["weights"].items():
            assert v == pytest.approx(res[0]["weights"][n], rel=1e-6, abs=1e-7)
