"""Elastic supervisor: keep a one-process-per-GPU training job running across lost nodes.

SURVEY §5 "Crash/OFFLINE": the reference defines ``NodeStatus.OFFLINE`` (trust_manager.py:18-23)
and a per-step training loop (distributed_trainer.py:324-352, 465-492) but nothing detects a dead
node or continues without it.  Here the pieces are:

1. every rank's heartbeat watchdog (``runtime/heartbeat.py``) marks a silent peer OFFLINE and, with
   ``abort_on_offline``, exits with code 17 instead of hanging inside the next RCCL collective;
2. this supervisor sees the generation fail, tells the LOST ranks from the collateral ones (the
   survivors' watchdogs report whom they saw go silent; without a report, ``blame`` ranks the exits
   of the ranks that went down together by severity), stops whatever is
   left (each worker is its own process group), and relaunches the job on the survivors only —
   one rank fewer per lost node, their GPUs dropped from ``HIP_VISIBLE_DEVICES``;
3. the relaunch resumes from the newest COMPLETE checkpoint (``utils/checkpoint.latest_checkpoint``):
   ``load_checkpoint`` re-plans the saved layers over the smaller world, broadcasts the plan and
   rebuilds each stage from the saved shards (weights, AdamW moments, verifier baselines, trust and
   detector state), and the trainer continues at the saved epoch / batch.

The supervisor is launcher-agnostic (it starts ``python -m trustworthy_dl.cli ...`` workers with
the torchrun environment contract: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT) and
never exec()s: workers are children, and the supervisor exits with the job's code.

    trustworthy-dl-elastic --nproc 8 --min-nproc 4 --max-restarts 3 -- --config configs/gpt2.yaml
"""
from __future__ import annotations

import argparse
import glob
import json
import logging
import os
import shutil
import signal
import socket
import subprocess
import sys
import tempfile
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

logger = logging.getLogger(__name__)

ABORT_CODE = 17  # heartbeat.py: a survivor that saw a peer go OFFLINE


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


HARD_DEATHS = {-9, -11, -7, -4, -8, 137, 139, 135, 132}  # SIGKILL/SEGV/BUS/ILL/FPE (signal or shell code)
COLLATERAL = {ABORT_CODE, -6, 134}                      # heartbeat abort; SIGABRT of a comm library


def blame(codes: Dict[int, int]) -> List[int]:
    """The lost ranks among those that went down together (``codes``: rank -> exit code, all within
    the first-failure window).  A dead peer takes its partners down within milliseconds (a gloo
    connection reset aborts them; RCCL survivors hang until the heartbeat watchdog aborts them with
    code 17), so exit ORDER cannot separate cause from collateral; severity does: a hard death
    (SIGKILL: OOM killer / lost host, SIGSEGV, SIGBUS...) outranks an ordinary error exit, which
    outranks the collateral kinds (code 17, SIGABRT)."""
    for tier in (lambda c: c in HARD_DEATHS, lambda c: c not in COLLATERAL, lambda c: c != ABORT_CODE):
        picked = sorted(r for r, c in codes.items() if tier(c))
        if picked:
            return picked
    return []


def node_ids_from_env(world: int) -> List[int]:
    """Physical identity of each rank of this generation: the original (generation-0) rank of the
    node now running as rank i (TDL_ELASTIC_NODE_IDS, set by the supervisor; identity otherwise).
    Checkpoints record it so a resume on survivors re-attaches trust / detection state to the same
    physical nodes, whichever ranks were lost (utils/checkpoint._resize_trust)."""
    raw = os.environ.get("TDL_ELASTIC_NODE_IDS", "")
    try:
        ids = [int(x) for x in raw.split(",") if x.strip()]
    except ValueError:
        ids = []
    return ids if len(ids) == world else list(range(world))


def default_devices(nproc: int, env: Optional[Dict[str, str]] = None) -> Optional[List[str]]:
    """GPU list when --devices is not given: the inherited HIP_VISIBLE_DEVICES, else 0..nproc-1 on a
    host with GPUs (so that dropping a lost rank drops ITS GPU, not the last one); None without GPUs
    (CPU / gloo jobs)."""
    env = os.environ if env is None else env
    vis = env.get("HIP_VISIBLE_DEVICES") or env.get("ROCR_VISIBLE_DEVICES") or env.get("CUDA_VISIBLE_DEVICES")
    if vis:
        devs = [d.strip() for d in vis.split(",") if d.strip()]
        if len(devs) >= nproc:
            return devs[:nproc]
    if os.path.exists("/dev/kfd") and glob.glob("/dev/dri/renderD*"):
        return [str(i) for i in range(nproc)]
    return None


@dataclass
class Generation:
    index: int
    world: int
    devices: Optional[List[str]]
    node_ids: List[int] = field(default_factory=list)
    exit_codes: Dict[int, Optional[int]] = field(default_factory=dict)
    lost: List[int] = field(default_factory=list)
    wall_s: float = 0.0
    ok: bool = False


class ElasticSupervisor:
    def __init__(self, train_args: List[str], nproc: int, min_nproc: int = 1, max_restarts: int = 3,
                 devices: Optional[List[str]] = None, grace_s: float = 60.0, timeout_s: Optional[float] = None,
                 env: Optional[Dict[str, str]] = None, python: str = sys.executable, log_dir: Optional[str] = None):
        self.train_args = list(train_args)
        self.nproc, self.min_nproc, self.max_restarts = nproc, max(1, min_nproc), max_restarts
        self.env = dict(os.environ if env is None else env)
        self.devices = list(devices) if devices else default_devices(nproc, self.env)
        self.grace_s, self.timeout_s = grace_s, timeout_s
        self.window_s = 2.0  # exits this close to the first one count as "went down together"
        self.python = python
        self.log_dir = log_dir
        self.generations: List[Generation] = []

    # ------------------------------------------------------------------ one generation
    def _cmd(self, gen: int) -> List[str]:
        args = list(self.train_args)
        if "--abort-on-offline" not in args:
            args.append("--abort-on-offline")
        if gen > 0:
            # a restart resumes from the newest complete checkpoint — including those the failed
            # generation wrote — never from the user's original --resume path again
            out, i = [], 0
            while i < len(args):
                if args[i] == "--resume":
                    i += 2
                    continue
                if args[i].startswith("--resume="):
                    i += 1
                    continue
                out.append(args[i])
                i += 1
            args = out + ["--resume", "latest"]
        return [self.python, "-m", "trustworthy_dl.cli", *args]

    def _report_dir(self, g: Generation) -> str:
        base = self.log_dir or os.path.join(tempfile.gettempdir(), f"tdl_elastic_{os.getpid()}")
        return os.path.join(base, f"gen{g.index}.reports")

    def _reports(self, g: Generation) -> Dict[int, List[int]]:
        out = {}
        d = self._report_dir(g)
        for r in range(g.world):
            f = os.path.join(d, f"offline.rank{r}.json")
            if os.path.exists(f):
                try:
                    with open(f) as fh:
                        out[r] = [int(x) for x in json.load(fh)]
                except (OSError, ValueError):
                    pass
        return out

    def _spawn(self, g: Generation) -> List[subprocess.Popen]:
        port = _free_port()
        procs = []
        rdir = self._report_dir(g)
        shutil.rmtree(rdir, ignore_errors=True)
        for r in range(g.world):
            env = dict(self.env)
            env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(g.world), "LOCAL_WORLD_SIZE": str(g.world),
                        "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                        "TDL_ELASTIC_GENERATION": str(g.index), "TDL_ELASTIC_RESTARTS": str(g.index),
                        "TDL_ELASTIC_REPORT_DIR": rdir,
                        "TDL_ELASTIC_NODE_IDS": ",".join(str(n) for n in (g.node_ids or range(g.world)))})
            if g.devices is not None:
                env["HIP_VISIBLE_DEVICES"] = ",".join(g.devices)
            out = None
            if self.log_dir:
                os.makedirs(self.log_dir, exist_ok=True)
                out = open(os.path.join(self.log_dir, f"gen{g.index}.rank{r}.log"), "w")
            procs.append(subprocess.Popen(self._cmd(g.index), env=env, stdout=out or None,
                                          stderr=subprocess.STDOUT if out else None, start_new_session=True))
            if out:
                out.close()
        return procs

    @staticmethod
    def _stop(procs: List[subprocess.Popen]):
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGTERM)
                except ProcessLookupError:
                    pass
        t0 = time.monotonic()
        for p in procs:
            try:
                p.wait(timeout=max(0.1, 10.0 - (time.monotonic() - t0)))
            except subprocess.TimeoutExpired:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()

    def _run_generation(self, g: Generation) -> Generation:
        t0 = time.monotonic()
        procs = self._spawn(g)
        first_fail = None
        exit_at: Dict[int, float] = {}
        try:
            while True:
                codes = [p.poll() for p in procs]
                now = time.monotonic()
                for r, c in enumerate(codes):
                    if c is not None and r not in exit_at:
                        exit_at[r] = now
                if all(c == 0 for c in codes):
                    g.ok = True
                    break
                failed = [r for r, c in enumerate(codes) if c not in (None, 0)]
                if failed and first_fail is None:
                    first_fail = now
                    logger.error("elastic: generation %d: rank(s) %s exited (%s); waiting up to %.0fs for the "
                                 "survivors to notice", g.index, failed, [codes[r] for r in failed], self.grace_s)
                if first_fail is not None and (all(c is not None for c in codes)
                                               or time.monotonic() - first_fail > self.grace_s):
                    break
                if self.timeout_s is not None and time.monotonic() - t0 > self.timeout_s:
                    logger.error("elastic: generation %d timed out after %.0fs", g.index, self.timeout_s)
                    break
                time.sleep(0.2)
            alive = [r for r, p in enumerate(procs) if p.poll() is None]
        finally:
            self._stop(procs)
        g.exit_codes = {r: p.returncode for r, p in enumerate(procs)}
        if not g.ok and first_fail is not None:
            near = {r: g.exit_codes[r] for r, t in exit_at.items() if t <= first_fail + self.window_s
                    and g.exit_codes[r] not in (None, 0)}
            reports = self._reports(g)
            voted = sorted({n for offs in reports.values() for n in offs if n not in reports and 0 <= n < g.world})
            if voted:
                # the survivors' heartbeat watchdogs saw these ranks go silent: the authoritative answer
                g.lost = voted
            else:
                g.lost = blame(near)
            if not voted and alive and all(c == ABORT_CODE for r, c in near.items()):
                # everyone who exited did so on purpose (heartbeat abort): the ranks still running
                # after the grace period are the silent ones — hung, not dead
                g.lost = alive
        # (a timeout with everyone alive blames nobody: restart at full size)
        g.wall_s = time.monotonic() - t0
        return g

    # ------------------------------------------------------------------ driver
    def run(self) -> Dict:
        world, devices, ids = self.nproc, self.devices, list(range(self.nproc))
        for gi in range(self.max_restarts + 1):
            g = self._run_generation(Generation(gi, world, devices, list(ids)))
            self.generations.append(g)
            logger.info("elastic: generation %d world %d -> %s (lost %s, %.1fs)", gi, world,
                        "ok" if g.ok else "failed", g.lost, g.wall_s)
            if g.ok:
                break
            survivors = [r for r in range(world) if r not in g.lost]
            if len(survivors) < self.min_nproc:
                logger.error("elastic: %d survivors < min %d: giving up", len(survivors), self.min_nproc)
                break
            if devices is not None:
                devices = [devices[r] for r in survivors]
            ids = [ids[r] for r in survivors]
            world = len(survivors)
        return self.summary()

    def summary(self) -> Dict:
        return {"ok": bool(self.generations and self.generations[-1].ok),
                "final_world": self.generations[-1].world if self.generations else 0,
                "generations": [{"gen": g.index, "world": g.world, "devices": g.devices, "node_ids": g.node_ids,
                                 "ok": g.ok, "lost": g.lost,
                                 "exit_codes": g.exit_codes, "wall_s": round(g.wall_s, 2)} for g in self.generations]}


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    train_args: List[str] = []
    if "--" in argv:
        i = argv.index("--")
        argv, train_args = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser(description="elastic one-process-per-GPU launcher with shrink-on-failure")
    ap.add_argument("--nproc", type=int, required=True)
    ap.add_argument("--min-nproc", type=int, default=1)
    ap.add_argument("--max-restarts", type=int, default=3)
    ap.add_argument("--devices", type=str, default=None,
                    help="comma list of GPU ids (default: the inherited HIP_VISIBLE_DEVICES, else 0..nproc-1 on GPU hosts)")
    ap.add_argument("--grace", type=float, default=60.0, help="seconds the survivors get to abort after a loss")
    ap.add_argument("--log-dir", type=str, default=None)
    ap.add_argument("--summary", type=str, default=None, help="write the generation summary JSON here")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    devices = a.devices.split(",") if a.devices else None
    sup = ElasticSupervisor(train_args, a.nproc, a.min_nproc, a.max_restarts, devices=devices, grace_s=a.grace,
                            log_dir=a.log_dir)
    res = sup.run()
    print(json.dumps(res), flush=True)
    if a.summary:
        with open(a.summary, "w") as f:
            json.dump(res, f, indent=2)
    return 0 if res["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
