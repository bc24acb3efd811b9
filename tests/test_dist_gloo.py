"""Multi-process pipeline correctness on CPU/gloo (BASELINE config 1: ResNet-32 CIFAR-10 2-stage MP).

The distributed 1F1B engine (one process per stage, P2P activations / grads) must reproduce the
single-process run: same losses step by step and same final weights."""
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


def _make_batches(model_name, n, bs):
    g = torch.Generator().manual_seed(42)
    out = []
    for _ in range(n):
        if model_name.startswith("gpt2"):
            ids = torch.randint(0, 1000, (bs, 33), generator=g)
            out.append({"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()})
        else:
            out.append({"input": torch.randn(bs, 3, 32, 32, generator=g), "target": torch.randint(0, 10, (bs,), generator=g)})
    return out


def _build(model_name, nodes, micro, p2p_mode="async", granularity="auto"):
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.flat import AdamWConfig
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    kw = {"seq_len": 32} if model_name.startswith("gpt2") else {}
    if model_name.startswith("gpt2"):
        kw["vocab_size"] = 1024
    m = get_model(model_name, seed=7, **kw)
    cfg = EngineConfig(num_nodes=nodes, micro_batches=micro, device="cpu", seq_len=32, p2p_mode=p2p_mode,
                       layer_granularity=granularity, adamw=AdamWConfig(lr=1e-2, eps=1.0, max_grad_norm=float(os.environ.get("TDL_TEST_CLIP", "1.0"))),
                       reassign=False)
    from trustworthy_dl.utils.metrics import MetricsCollector
    return PipelineEngine(m, cfg, metrics=MetricsCollector())


def _worker(rank, world, port, model_name, steps, micro, out_path, p2p_mode="async", granularity="auto"):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = _build(model_name, world, micro, p2p_mode, granularity)
    clip = []
    for b in _make_batches(model_name, steps, 8):
        eng.train_step(b)
        clip.append(float(eng.my_stage().verifier.ctrl[0]))
    eng.flush()
    st = eng.stage_state_dicts()
    res = {"rank": rank, "last_loss": eng.last_loss, "losses": [m["loss"] for m in eng.metrics.batch_metrics],
           "weights": {n: float(t.double().sum()) for sd in st.values() for n, t in sd.items()},
           "trust": [eng.trust.get_trust_score(i) for i in range(world)], "clip": clip}
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("model_name,micro,world,p2p,gran", [
    ("resnet32", 2, 2, "async", "auto"), pytest.param("gpt2-tiny", 4, 2, "async", "auto", marks=pytest.mark.slow),
    ("gpt2-tiny", 4, 2, "grouped", "auto"),
    pytest.param("gpt2-tiny", 2, 4, "async", "auto", marks=pytest.mark.slow),
    pytest.param("gpt2-tiny", 8, 4, "async", "auto", marks=pytest.mark.slow),
    ("gpt2-tiny", 4, 4, "async", "half")])  # stage boundaries inside blocks, one process per stage
def test_pipeline_matches_single_process(model_name, micro, world, p2p, gran, monkeypatch):
    steps = 4
    if model_name.startswith("gpt2"):
        monkeypatch.setenv("TDL_TEST_CLIP", "0.05")  # clipping binds on every step
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "res")
        mp.spawn(_worker, args=(world, _free_port(), model_name, steps, micro, out, p2p, gran), nprocs=world, join=True)
        res = [json.load(open(f"{out}.{r}")) for r in range(world)]
    torch.set_num_threads(4)
    local = _build(model_name, world, micro, granularity=gran)
    for b in _make_batches(model_name, steps, 8):
        local.train_step(b)
    local.flush()
    # losses agree (the loss is produced on the last stage and gathered to every rank); the first
    # step is before any update (bitwise-close), later steps differ only by fp32 summation order
    ref_losses = [m["loss"] for m in local.metrics.batch_metrics]
    for r in range(world):
        assert res[r]["losses"][0] == pytest.approx(ref_losses[0], rel=1e-5)
        assert res[r]["losses"] == pytest.approx(ref_losses, rel=2e-3)
    # weights agree stage by stage (eps=1 keeps the AdamW update linear in the gradient, so fp32
    # summation-order noise is not amplified into sign flips of near-zero gradient entries)
    lw = local.stage_state_dicts()
    for r in range(world):
        for n, v in res[r]["weights"].items():
            ref = float(lw[r][n].double().sum())
            assert v == pytest.approx(ref, rel=1e-4, abs=1e-5), (r, n)
    # every rank holds the same trust vector (identical all-gathered digests)
    for r in range(1, world):
        assert res[0]["trust"] == pytest.approx(res[r]["trust"])
    if model_name.startswith("gpt2"):
        # ... and the pipeline depth does not change the training trajectory: the same model on ONE
        # stage (global-norm clipping on, the tied wte counted once) gives the same losses
        single = _build(model_name, 1, micro, granularity="block")
        clip1 = []
        for b in _make_batches(model_name, steps, 8):
            single.train_step(b)
            clip1.append(float(single.stages[0].verifier.ctrl[0]))
        single.flush()
        one = [m["loss"] for m in single.metrics.batch_metrics]
        assert res[0]["losses"] == pytest.approx(one, rel=1e-4), (res[0]["losses"], one)
        # the global clip scale (from the all-gathered per-stage sums of squares) is the one-stage scale
        assert max(clip1) < 0.99, "clipping must bind for this check"
        for r in range(world):
            assert res[r]["clip"] == pytest.approx(clip1, rel=1e-4), (r, res[r]["clip"], clip1)


def _layer_sums(eng):
    return {li: float(eng._pack_layer(st, li).double().sum())
            for st in eng.stages.values() for li in range(*st.layer_range)}


def _reshard_run(eng, batches, rank_is_tampered):
    for b in batches[:4]:
        eng.train_step(b)
    eng.flush()
    if rank_is_tampered:
        with torch.no_grad():
            eng.stages[1].flat.master.add_(1000.0)      # node 1 scribbles over its own weights
    eng.reassign([1], step=eng.global_step)
    rec = eng.reassignment_history[-1]
    for b in batches[4:]:
        eng.train_step(b)
    eng.flush()
    return rec


def _reshard_worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = _build("gpt2-tiny", world, 2)
    eng.cfg.shadow_interval = 2
    rec = _reshard_run(eng, _make_batches("gpt2-tiny", 6, 8), rank == 1)
    res = {"rank": rank, "sums": _layer_sums(eng), "restored": {str(k): v for k, v in rec["restored_from_shadow"].items()},
           "plan": eng.plan.ranks, "last_loss": eng.last_loss, "link_measured": eng.link_meter.measured(),
           "link_bw": eng.link_meter.bytes_per_s(), "est": rec["estimated_migration_time"],
           "moved": rec["moved_params"], "actual": rec["migration_time"], "phases": rec["phases"]}
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump(res, f)
    dist.barrier()
    dist.destroy_process_group()


def test_distributed_reshard_restores_from_shadow_and_matches_local():
    """Re-shard mid-training over gloo (3 stages -> 2): node 1 is excluded, its layers are rebuilt
    from the snapshot node 2 holds (its own memory was tampered with), training continues, and the
    final per-layer state equals the single-process run of the same sequence."""
    world = 3
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "res")
        mp.spawn(_reshard_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = [json.load(open(f"{out}.{r}")) for r in range(world)]
    eng = _build("gpt2-tiny", world, 2)
    eng.cfg.shadow_interval = 2
    rec = _reshard_run(eng, _make_batches("gpt2-tiny", 6, 8), True)
    ref = _layer_sums(eng)
    got = {}
    for r in res:
        assert r["restored"] == {"1": 4} and r["plan"] == [0, 2]
        # the migration estimate uses this job's measured transfers (shadow snapshots), not the
        # prior, plus the rebuild / pack terms calibrated on the engine's own build; it is a
        # prediction made before the move, compared with the measured wall time
        assert r["link_measured"] and r["link_bw"] != 2e9
        assert r["est"] >= r["moved"] * 12 / r["link_bw"]
        assert set(r["phases"]) >= {"pack_s", "transfer_s", "rebuild_s", "groups_s", "unpack_s"}
        print("reshard est/actual", r["rank"], r["est"], r["actual"], r["phases"])
        got.update({int(k): v for k, v in r["sums"].items()})
    assert rec["restored_from_shadow"] == {1: 4}
    assert sorted(got) == sorted(ref)
    for li in ref:
        assert abs(got[li] - ref[li]) <= 1e-4 * max(1.0, abs(ref[li])), (li, got[li], ref[li])
    assert max(abs(v) for v in ref.values()) < 1e6
    assert res[0]["last_loss"] is not None and abs(res[0]["last_loss"] - eng.last_loss) < 1e-3


def _replan_worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = _build("gpt2-tiny", world, 2)
    batches = _make_batches("gpt2-tiny", 6, 4)
    inv = [eng.comm_inventory()]
    eng.train_step(batches[0])
    eng.flush()
    eng.reassign([world - 1], 1)              # re-shard away from the last rank: a new tie group
    inv.append(eng.comm_inventory())
    for i in range(3):                         # three more re-plans onto member sets seen before
        eng._build()
        eng.train_step(batches[1 + i])
        eng.flush()
        inv.append(eng.comm_inventory())
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump({"inv": inv, "loss": eng.last_loss}, f)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
def test_replans_reuse_process_groups():
    """Re-plans do not leak communicators: groups are cached by member set, so re-planning onto a
    member set seen before creates nothing; each rank's communicator and stream counts stay bounded
    and within the 32 hardware queues (verdict r2: every _build created new tie / DP groups)."""
    world = 4
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "inv")
        mp.spawn(_replan_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        res = [json.load(open(f"{out}.{r}")) for r in range(world)]
    for r in res:
        created = [i["groups_created"] for i in r["inv"]]
        assert created[0] == 4                   # act + grad direction groups + audit group + tie group (0, 3)
        assert created[1] == 5                   # + tie group (0, 2) after the re-shard
        assert created[2:] == [5, 5, 5]          # re-plans onto known member sets reuse them
        assert all(i["hip_streams"] <= 32 for i in r["inv"])
        assert r["inv"][-1]["rccl_comms"] == r["inv"][1]["rccl_comms"]
        assert r["loss"] is not None
