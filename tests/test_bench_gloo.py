"""bench.py contract under the multi-rank launcher (gloo on CPU, tiny GPT-2): the driver runs
``torch.distributed.run --nproc-per-node N bench.py --gpus N`` and parses ONE JSON line from rank 0.

Covers 2 / 4 / 8 ranks in both pipeline P2P modes, a mid-run re-shard (--reassign-at), and the
failure path: a rank that hangs or raises must turn into one failure JSON line from rank 0 naming
the phase of every rank, and a non-zero exit, well before any collective time-out."""
import json
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(n, *extra, model="gpt2-tiny", timeout=300):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "2", "--warmup", "1",
           "--model", model, "--seq-len", "32", "--batch-per-gpu", "4", *extra]
    t0 = time.time()
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    return out, lines, time.time() - t0


@pytest.mark.parametrize("n,mode", [(2, "async"), (2, "grouped"), (4, "async"), (4, "grouped"),
                                    (8, "async"), (8, "grouped")])
@pytest.mark.slow
def test_bench_multirank_json_line(n, mode):
    model = "gpt2-mini" if n == 8 else "gpt2-tiny"   # gpt2-tiny has fewer pipeline units than 8
    out, lines, _ = _run(n, "--p2p-mode", mode, model=model)
    assert out.returncode == 0, out.stderr[-3000:]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["steps"] == 2 and d["warmup"] == 1
    assert d["config"]["global_batch"] == 4 * n and d["config"]["parallelism"] == f"pp{n}"
    assert d["value"] > 0 and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["config"]["last_loss"] is not None
    assert d["config"]["p2p_mode"] == mode and d["config"]["p2p_mode_requested"] == mode
    assert len(d["config"]["hw_queues_per_rank"]) == n
    assert out.stderr.count("GPU_MAX_HW_QUEUES=") == n        # every rank logs its queue setting
    # communicator / stream inventory per rank: interior stages talk to 2 neighbours, end stages to 1
    comms, streams = d["config"]["rccl_comms_per_rank"], d["config"]["hip_streams_per_rank"]
    assert len(comms) == n and len(streams) == n
    per_peer = 2 if mode == "async" else 1            # async: one activation + one gradient communicator per peer
    groups = (2 if mode == "async" else 0) + 1        # the two direction groups + the audit group
    tie = 1                                           # the tied embedding / LM head all-reduce group
    ranks = [int(x.split("@rank")[1].split(":")[0]) for x in d["config"]["plan"].split() if "@rank" in x]
    for r, c in enumerate(comms):
        if r not in ranks:                            # idle rank (fewer pipeline units than ranks)
            assert c == 1 + groups and streams[r] == c + 1, (r, comms, streams)
            continue
        i = ranks.index(r)
        S = len(ranks)
        nb = ({i - 1} if i > 0 else set()) | ({i + 1} if i < S - 1 else set())
        # trusted weight snapshots (taken at build time and every shadow_interval steps) travel on
        # the default group to the next min(2, S - 1) stages of the ring, and in from the previous ones
        k = min(2, S - 1)
        ring = {(i + dd) % S for dd in range(1, k + 1)} | {(i - dd) % S for dd in range(1, k + 1)}
        default_peers = (ring | nb) if mode == "grouped" else ring
        dir_peers = nb if mode == "async" else set()
        # mirror-mode audit on its own group: applied gradient / openings to the auditor (next stage,
        # or the previous one for the loss stage), the same from the auditee
        audit_peers = nb
        expect = 1 + groups + (tie if i in (0, S - 1) else 0) + 2 * len(dir_peers) + len(default_peers) \
            + len(audit_peers)
        assert c == expect, (r, comms, expect)
        assert streams[r] == c + 2                    # + compute stream + verification side stream
    assert max(streams) <= 32


@pytest.mark.slow
def test_bench_midrun_reassign():
    out, lines, _ = _run(4, "--reassign-at", "2")
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads(lines[0])
    (r,) = d["config"]["reassignments"]
    assert r["from_nodes"] == [3] and r["step"] == 2
    assert "@rank3" not in r["plan"] and r["plan"].count("stage") == 3
    assert d["config"]["last_loss"] is not None and d["value"] > 0
    # the re-plan reused the direction and audit groups and created ONE new tie group (ranks 0 and 2)
    assert d["config"]["process_groups_created"] == 2 + 1 + 1 + 1


@pytest.mark.slow
@pytest.mark.parametrize("fault", ["hang", "raise"])
def test_bench_failure_is_legible(fault):
    out, lines, wall = _run(4, "--watchdog", "8", "--debug-fault", fault, "--debug-fault-rank", "2",
                            "--debug-fault-step", "1", timeout=200)
    assert out.returncode != 0
    assert len(lines) == 1, (out.stdout[-2000:], out.stderr[-2000:])
    d = json.loads(lines[0])
    assert d["value"] is None and d["failure_kind"] == ("stall" if fault == "hang" else "error")
    assert "injected" in d["failed_phase"]["2"]
    if fault == "hang":
        assert "rank 2" in d["error"] or any("rank 2" in p for p in d["failed_phase"].values())
    else:
        assert d["errors"][0]["rank"] == 2 and "injected fault" in d["errors"][0]["error"]
    assert wall < 150
