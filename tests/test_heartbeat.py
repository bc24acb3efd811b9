"""Heartbeat watchdog -> NodeStatus.OFFLINE (and back), agreed on by every rank through the digest."""
import json
import os
import socket
import tempfile
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_monitor_detects_silence_and_recovery():
    from trustworthy_dl.runtime.heartbeat import HeartbeatMonitor
    store = dist.HashStore()
    a = HeartbeatMonitor(store, 0, 2, interval=0.05, timeout=0.3)
    b = HeartbeatMonitor(store, 1, 2, interval=0.05, timeout=0.3)
    seen = []
    a.on_offline = lambda n: seen.append(("off", n))
    a.on_online = lambda n: seen.append(("on", n))
    a.start(), b.start()
    time.sleep(0.4)
    assert a.offline() == set()
    b.pause()
    time.sleep(0.8)
    assert a.offline() == {1}
    b.resume()
    time.sleep(0.4)
    assert a.offline() == set()
    a.stop(), b.stop()
    assert seen == [("off", 1), ("on", 1)]


def _worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    m = get_model("gpt2-tiny", seed=3, seq_len=16, vocab_size=256)
    eng = PipelineEngine(m, EngineConfig(num_nodes=world, micro_batches=2, device="cpu", seq_len=16, reassign=False,
                                         heartbeat_interval=0.05, heartbeat_timeout=0.3))
    g = torch.Generator().manual_seed(0)
    ids = torch.randint(0, 256, (4, 17), generator=g)
    batch = {"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()}
    statuses = []
    for step in range(6):
        if rank == 0 and step == 2:
            eng.heartbeat.pause()   # rank 0's process "hangs" (its training loop still runs here)
        if rank == 0 and step == 4:
            eng.heartbeat.resume()
        time.sleep(0.6 if step in (2, 4) else 0.0)
        eng.train_step(batch)
        eng.flush()
        statuses.append(eng.trust.get_node_status(0).value)
    eng.close()
    with open(f"{out_path}.{rank}", "w") as f:
        json.dump({"status": statuses, "events": eng.node_events}, f)
    dist.barrier()
    dist.destroy_process_group()


def test_offline_agreed_by_all_ranks_and_recovers():
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "res")
        mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
        res = [json.load(open(f"{out}.{r}")) for r in range(2)]
    # rank 1's watchdog sees rank 0 silent during steps 2-3; both ranks adopt OFFLINE from the digest
    assert res[0]["status"] == res[1]["status"]
    assert "offline" in res[0]["status"]
    assert res[0]["status"][-1] in ("recovering", "trusted", "suspicious")
    kinds = [e["event"] for e in res[0]["events"] if e["node_id"] == 0]
    assert kinds[:2] == ["offline", "online"]


class _DeadStore:
    def add(self, key, v):
        raise RuntimeError("Connection reset by peer (store host gone)")


def test_store_host_loss_marks_rank0_offline():
    """rank 0 hosts the TCPStore: when it dies every survivor's beat/poll fails.  Consecutive store
    failures for longer than the timeout declare the store host OFFLINE (survivors used to
    swallow the errors and never report anyone)."""
    from trustworthy_dl.runtime.heartbeat import HeartbeatMonitor
    m = HeartbeatMonitor(_DeadStore(), rank=2, world=3, interval=0.01, timeout=0.5)
    seen = []
    m.on_offline = seen.append
    m.store_failed(RuntimeError("x"), now=10.0)   # starts the clock
    m.store_failed(RuntimeError("x"), now=10.3)
    assert m.offline() == set()
    m.store_failed(RuntimeError("x"), now=10.6)
    assert m.offline() == {0} and seen == [0]
    m.store_failed(RuntimeError("x"), now=11.0)   # reported once
    assert seen == [0]
    # the store host itself never declares itself offline
    h = HeartbeatMonitor(_DeadStore(), rank=0, world=3, timeout=0.1)
    h.store_failed(RuntimeError("x"), now=0.0)
    h.store_failed(RuntimeError("x"), now=5.0)
    assert h.offline() == set()
