"""RCCL-model replay of the recorded communication (trustworthy_dl/runtime/commcheck.py).

The multi-rank CPU tests run on gloo, which is more permissive than RCCL (per-communicator issue
order, group semantics, stream-ordered waits).  Each bench schedule below runs on gloo with the
recorder on, then is replayed under the RCCL model: no operation may stay blocked and every send /
receive / collective must pair with an equal-sized partner."""
import os
import subprocess
import sys
import tempfile

import pytest

from trustworthy_dl.runtime.commcheck import replay, replay_dir

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _p2p(i, pg, *ops):
    return {"id": i, "kind": "p2p", "pg": pg, "ops": [list(o) for o in ops]}


def test_replay_finds_head_of_line_deadlock():
    """Both ranks queue a send ahead of the receive on ONE communicator, as separate operations:
    fine on gloo (its sends do not wait for the receive), a hang under RCCL."""
    ev = {0: [_p2p(0, "w", ("send", 1, 64)), _p2p(1, "w", ("recv", 1, 64))],
          1: [_p2p(0, "w", ("send", 0, 64)), _p2p(1, "w", ("recv", 0, 64))]}
    res = replay(ev)
    assert not res["ok"] and res["completed"] == 0 and len(res["blocked"]) == 2


def test_replay_batched_exchange_and_direction_communicators_are_fine():
    # the same exchange as ONE group: starts together, completes
    ev = {0: [_p2p(0, "w", ("send", 1, 64), ("recv", 1, 64))],
          1: [_p2p(0, "w", ("recv", 0, 64), ("send", 0, 64))]}
    assert replay(ev)["ok"]
    # separate communicators per direction (the async 1F1B design): no head-of-line blocking
    ev = {0: [_p2p(0, "act", ("send", 1, 64)), _p2p(1, "grad", ("recv", 1, 64))],
          1: [_p2p(0, "grad", ("send", 0, 64)), _p2p(1, "act", ("recv", 0, 64))]}
    assert replay(ev)["ok"]


def test_replay_wait_orders_communicators():
    """A rank that waits on a receive before issuing its send makes the send depend on it; a cycle
    through two communicators is a deadlock."""
    ev = {0: [_p2p(0, "a", ("recv", 1, 8)), {"wait": 0}, _p2p(1, "b", ("send", 1, 8))],
          1: [_p2p(0, "b", ("recv", 0, 8)), {"wait": 0}, _p2p(1, "a", ("send", 0, 8))]}
    assert not replay(ev)["ok"]


def test_replay_store_reveal_and_host_sync():
    """wait() is stream-ordered (the host goes on), so a store set after it is reached; a HOST sync
    before the set blocks the host until the receive completes, and the receive's sender issues its
    send only after reading the key: a cross-host deadlock."""
    ev = {0: [_p2p(0, "a", ("recv", 1, 8)), {"wait": 0}, {"store_set": "k"}],
          1: [{"store_get": "k"}, _p2p(0, "a", ("send", 0, 8))]}
    assert replay(ev)["ok"]
    ev[0] = [_p2p(0, "a", ("recv", 1, 8)), {"wait": 0}, {"host_sync": True}, {"store_set": "k"}]
    res = replay(ev)
    assert not res["ok"] and {b["rank"] for b in res["blocked"]} == {0, 1}


def test_replay_flags_size_and_count_mismatch():
    ev = {0: [_p2p(0, "w", ("send", 1, 64))], 1: [_p2p(0, "w", ("recv", 0, 32))]}
    res = replay(ev)
    assert not res["ok"] and res["mismatches"]
    ev = {0: [{"id": 0, "kind": "coll", "name": "all_reduce", "pg": "w", "bytes": 8, "members": [0, 1]}],
          1: [{"id": 0, "kind": "coll", "name": "broadcast", "pg": "w", "bytes": 8, "members": [0, 1]}]}
    assert replay(ev)["mismatches"]


def _bench(n, d, *extra, model="gpt2-tiny"):
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="1", TDL_COMMCHECK=d)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--steps", "2", "--warmup", "1", "--model", model, "--seq-len", "32",
           "--batch-per-gpu", "4", *extra]
    return subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)


@pytest.mark.parametrize("n,extra", [
    (2, ("--p2p-mode", "async")), (4, ("--p2p-mode", "grouped")), (4, ("--p2p-mode", "async", "--reassign-at", "2")),
    (4, ("--p2p-mode", "async", "--audit-targeted")),
    (8, ("--p2p-mode", "async")), (8, ("--p2p-mode", "grouped"))])
@pytest.mark.slow
def test_bench_schedule_replays_under_rccl_model(n, extra):
    """The bench's whole run (build-time shadows, 1F1B, forward + backward audit with its store
    reveal, digest all-gathers, tied all-reduce, re-shard) recorded on gloo and replayed under the
    RCCL model: nothing blocks, every operation pairs."""
    with tempfile.TemporaryDirectory() as d:
        out = _bench(n, d, *extra, model="gpt2-mini" if n == 8 else "gpt2-tiny")
        assert out.returncode == 0, out.stderr[-3000:]
        assert sorted(os.listdir(d)) == sorted(f"rank{r}.json" for r in range(n))
        res = replay_dir(d)
    assert res["ok"], res
    assert res["ops"] > 20 * n
