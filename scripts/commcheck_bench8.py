#!/usr/bin/env python3
"""The MP = 8 headline path rehearsed without 8 GPUs: bench.py on 8 gloo ranks (one process per
stage, GPT-2-medium layers at T = 32, audit protocol on: commitments, key / sketches / opening via the
c10d store, applied-gradient + opened-contribution P2P, live optimizer mirrors), with a mid-run
re-shard, every communication recorded (TDL_COMMCHECK) and replayed under the RCCL model
(runtime/commcheck.py: per-communicator issue order, grouped P2P, stream-ordered waits, store
reveals).  Writes the bench's JSON line (per-rank audit bytes / memory in ``audit_per_rank``) and the
replay verdict.

    python scripts/commcheck_bench8.py --out profiles/r6_commcheck_bench8.json
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2-medium")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--reassign-at", type=int, default=2)
    ap.add_argument("--out", default="profiles/r6_commcheck_bench8.json")
    a = ap.parse_args()
    from trustworthy_dl.runtime.commcheck import replay_dir
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    with tempfile.TemporaryDirectory() as d:
        env = dict(os.environ, CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="1", TDL_COMMCHECK=d)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.n}",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
               "--gpus", str(a.n), "--steps", str(a.steps), "--warmup", "1", "--model", a.model, "--seq-len", "32",
               "--batch-per-gpu", "4", "--p2p-mode", "async", "--reassign-at", str(a.reassign_at)]
        out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=3000)
        if out.returncode != 0:
            print(out.stderr[-4000:])
            sys.exit(out.returncode)
        line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
        bench = json.loads(line)
        res = replay_dir(d)
    rec = {"what": f"bench.py on {a.n} gloo ranks ({a.model} layers, T=32), audit protocol on, re-shard at step "
                   f"{a.reassign_at}, replayed under the RCCL model", "replay": res, "bench": bench}
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    aud = bench["config"].get("audit_per_rank", [])
    print(json.dumps({"replay_ok": res.get("ok"), "ops": res.get("ops"),
                      "audit_bytes_per_step_per_rank": [r.get("bytes_per_step") for r in aud],
                      "audit_memory_bytes_per_rank": [r.get("memory_bytes") for r in aud],
                      "reassignments": bench["config"].get("reassignments")}))


if __name__ == "__main__":
    main()
