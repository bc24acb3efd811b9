"""Resume into a different world size (gloo, CPU): a 4-rank pipeline saves a sharded checkpoint,
a 3-rank job loads it — rank 0 re-plans the saved layers over the live ranks, broadcasts the plan,
each rank assembles its stages layer by layer from the saved shards — and training continues on
the same loss trajectory as the uninterrupted 4-rank run, with trust / detector state restored.
Also: a local-mode 4 -> 3 resume, and a missing shard refusing to load."""
import json
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

KW = dict(model_name="gpt2-tiny", seq_len=32, micro_batches=4, batch_size=8, device="cpu", compute_dtype="fp32",
          checkpoint_interval=0, seed=5, layer_granularity="half", learning_rate=1e-3, max_grad_norm=1.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batches(n):
    g = torch.Generator().manual_seed(11)
    out = []
    for _ in range(n):
        ids = torch.randint(0, 2000, (8, 33), generator=g)
        out.append({"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()})
    return out


def _trainer(nodes):
    from trustworthy_dl import DistributedTrainer
    return DistributedTrainer(num_nodes=nodes, **KW)


def _worker(rank, world, port, ckpt, out_path, phase, save_at, total):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    tr = _trainer(world)
    tr.setup_distributed_environment(rank, world, backend="gloo")
    tr.create_model_partitions()
    e = tr.engine
    batches = _batches(total)
    res = {"rank": rank}
    if phase == "save":
        for b in batches[:save_at]:
            e.train_step(b)
        path = tr.save_checkpoint(ckpt)
        res["trust_at_save"] = [tr.trust_manager.get_trust_score(i) for i in range(world)]
        res["detector_at_save"] = dict(tr.attack_detector.detection_stats)
        for b in batches[save_at:]:       # uninterrupted reference continuation
            e.train_step(b)
        e.flush()
        res["path"] = path
    else:
        tr.load_checkpoint(ckpt)
        res["step_after_load"] = e.global_step
        res["plan"] = e.plan.describe()
        res["num_stages"] = e.plan.num_stages
        res["trust_after_load"] = [tr.trust_manager.get_trust_score(i) for i in range(world)]
        res["detector_after_load"] = dict(tr.attack_detector.detection_stats)
        res["replan"] = [r for r in e.reassignment_history if r.get("event") == "resume_replan"]
        for b in batches[save_at:]:
            e.train_step(b)
        e.flush()
    res["losses"] = [m["loss"] for m in e.metrics.batch_metrics if m.get("loss") is not None]
    res["steps"] = [m["step"] for m in e.metrics.batch_metrics if m.get("loss") is not None]
    with open(f"{out_path}.{phase}.{rank}", "w") as f:
        json.dump(res, f, default=str)
    dist.barrier()
    tr.cleanup()


@pytest.mark.slow
def test_resume_4_ranks_into_3():
    total, save_at = 5, 3
    with tempfile.TemporaryDirectory() as d:
        ck = os.path.join(d, "ck", "checkpoint_step_3.pt")
        out = os.path.join(d, "res")
        mp.spawn(_worker, args=(4, _free_port(), ck, out, "save", save_at, total), nprocs=4, join=True)
        assert os.path.exists(ck) and all(os.path.exists(ck.replace(".pt", f".rank{r}.pt")) for r in range(4))
        mp.spawn(_worker, args=(3, _free_port(), ck, out, "resume", save_at, total), nprocs=3, join=True)
        saved = [json.load(open(f"{out}.save.{r}")) for r in range(4)]
        resumed = [json.load(open(f"{out}.resume.{r}")) for r in range(3)]
    ref = saved[0]
    r0 = resumed[0]
    assert all(r["step_after_load"] == save_at for r in resumed)
    assert r0["num_stages"] == 3 and all(r["plan"] == r0["plan"] for r in resumed)   # one broadcast plan
    assert r0["replan"] and r0["replan"][0]["step"] == save_at
    # the resumed 3-rank job continues the 4-rank trajectory (pipeline depth does not change the math)
    ref_tail = dict(zip(ref["steps"], ref["losses"]))
    got = dict(zip(r0["steps"], r0["losses"]))
    assert set(got) == set(range(save_at + 1, total + 1)), got
    for s, v in got.items():
        assert v == pytest.approx(ref_tail[s], rel=2e-4), (s, v, ref_tail[s])
    # trust + detector state restored (nodes beyond the live world are retired)
    assert r0["trust_after_load"] == pytest.approx(ref["trust_at_save"][:3])
    assert ref["detector_at_save"]["true_negatives"] > 0
    assert r0["detector_after_load"]["true_negatives"] == ref["detector_at_save"]["true_negatives"]


@pytest.mark.slow
def test_local_resume_4_into_3_and_missing_shard(tmp_path):
    from trustworthy_dl.utils.checkpoint import consolidate
    batches = _batches(4)
    a = _trainer(4)
    a.create_model_partitions()
    for b in batches[:2]:
        a.engine.train_step(b)
    path = a.save_checkpoint(str(tmp_path / "ck.pt"))
    for b in batches[2:]:
        a.engine.train_step(b)
    a.engine.flush()
    ref = {m["step"]: m["loss"] for m in a.metrics_collector.batch_metrics if m.get("loss") is not None}

    b3 = _trainer(3)
    b3.create_model_partitions()
    b3.load_checkpoint(path)
    assert b3.engine.plan.num_stages == 3 and b3.engine.global_step == 2
    for b in batches[2:]:
        b3.engine.train_step(b)
    b3.engine.flush()
    got = {m["step"]: m["loss"] for m in b3.metrics_collector.batch_metrics if m.get("loss") is not None}
    for s in (3, 4):
        assert got[s] == pytest.approx(ref[s], rel=2e-4)

    # a sharded manifest whose shard is gone must refuse to load
    ck = torch.load(path, weights_only=True)
    ck["shards"] = ["gone.rank0.pt"]
    bad = str(tmp_path / "bad.pt")
    torch.save(ck, bad)
    with pytest.raises(FileNotFoundError):
        consolidate(bad)
