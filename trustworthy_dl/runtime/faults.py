"""Deterministic fault injection for the failure-recovery tests and drills (SURVEY §5 "Crash/OFFLINE").

``TDL_FAULT_INJECT`` holds ``;``-separated faults ``kind:rank=R:step=S[:gen=G]``:

* ``crash`` — the process SIGKILLs itself right after optimizer step S (a node lost without any
  goodbye: its heartbeat stops, its sockets close mid-collective);
* ``hang``  — the process stops making progress (sleeps forever inside the step loop) while its
  heartbeat thread is paused too, as for a wedged host.

``gen`` restricts the fault to one generation of an elastic job (``TDL_ELASTIC_GENERATION``, set by
``runtime/elastic.py``; default 0), so a restarted job does not re-inject it.
"""
from __future__ import annotations

import logging
import os
import signal
import time
from typing import Dict, List

logger = logging.getLogger(__name__)


def parse(spec: str) -> List[Dict]:
    out = []
    for part in filter(None, (p.strip() for p in spec.split(";"))):
        kind, *kv = part.split(":")
        f = {"kind": kind, "rank": 0, "step": 0, "gen": 0}
        for item in kv:
            k, v = item.split("=")
            f[k] = int(v)
        if kind not in ("crash", "hang"):
            raise ValueError(f"unknown fault kind {kind!r} in TDL_FAULT_INJECT")
        out.append(f)
    return out


def generation() -> int:
    return int(os.environ.get("TDL_ELASTIC_GENERATION", "0"))


def maybe_inject(rank: int, step: int, heartbeat=None):
    spec = os.environ.get("TDL_FAULT_INJECT")
    if not spec:
        return
    gen = generation()
    for f in parse(spec):
        if f["rank"] != rank or f["step"] != step or f["gen"] != gen:
            continue
        logger.error("fault injection: %s on rank %d at step %d (generation %d)", f["kind"], rank, step, gen)
        if f["kind"] == "crash":
            os.kill(os.getpid(), signal.SIGKILL)
        else:
            if heartbeat is not None:
                heartbeat.pause()
            while True:
                time.sleep(3600)
