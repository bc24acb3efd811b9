"""Progress marks + a stall / failure watchdog for multi-rank runs (bench.py, the CLI trainer).

Every rank records where it is (``mark("step 3: stage 2 waits for a P2P receive from rank 1")``)
with a timestamp.  A daemon thread publishes the latest mark to the process group's TCP store every
``publish_s`` seconds (the store keeps working while an RCCL collective hangs).  Rank 0's thread
also reads every rank's mark and an error counter in the store, so that

* a rank that raises calls :meth:`StallWatchdog.report_error` (store key + counter) and waits a
  moment for rank 0 to acknowledge before exiting non-zero, and
* a rank (any rank) that has not advanced for ``stall_s`` seconds,

become ONE failure record handed to ``on_failure(kind, marks, errors)`` on rank 0 (bench.py prints
its failure JSON line there), after which rank 0 ends with ``exit_code``.  Non-zero ranks give rank
0 ``grace_s`` extra seconds before their own stall exit, so torchrun does not tear the job down
before the report is out.  Nothing here re-execs or signals other processes.

(SURVEY 5 "failure detection"; the reference's bring-up, /root/reference/distributed_trainer.py:99-114,
has no failure reporting: a hung collective there is a silent time-out of the whole job.)
"""
from __future__ import annotations

import datetime
import json
import os
import sys
import threading
import time
from typing import Callable, Dict, List, Optional

_state = {"phase": "start", "t": time.time(), "rank": 0}
_lock = threading.Lock()


def mark(phase: str) -> None:
    with _lock:
        _state["phase"] = phase
        _state["t"] = time.time()


def current() -> Dict:
    with _lock:
        return dict(_state)


_ERR_COUNT = "tdl/errors"
_ERR_KEY = "tdl/error/{}"
_ACK = "tdl/error_reported"
_PROG = "tdl/progress/{}"


class StallWatchdog:
    def __init__(self, rank: int, world: int, stall_s: float, store=None,
                 on_failure: Optional[Callable[[str, Dict[int, Dict], List[Dict]], None]] = None,
                 publish_s: float = 1.0, exit_code: int = 3, grace_s: float = 15.0):
        self.rank, self.world = rank, world
        self.stall_s = float(stall_s)
        self.store = store
        self.on_failure = on_failure
        self.publish_s = publish_s
        self.exit_code = exit_code
        self.grace_s = grace_s
        self._stop = threading.Event()
        self._fired = threading.Lock()
        with _lock:
            _state["rank"] = rank
        self._thread = threading.Thread(target=self._run, name="tdl-stall-watchdog", daemon=True)

    def start(self) -> "StallWatchdog":
        self._publish(current())
        if self.stall_s > 0 or (self.rank == 0 and self.store is not None):
            self._thread.start()
        return self

    def stop(self) -> None:
        self._stop.set()

    # ------------------------------------------------------------------ store helpers
    def _publish(self, st: Dict) -> None:
        if self.store is None:
            return
        try:
            self.store.set(_PROG.format(self.rank), json.dumps(st))
        except Exception:  # noqa: BLE001 - the store may be gone during teardown
            pass

    def _get(self, key: str):
        try:
            if not self.store.check([key]):
                return None
            return self.store.get(key)
        except Exception:  # noqa: BLE001
            return None

    def snapshot(self) -> Dict[int, Dict]:
        """Latest mark of every rank (own from memory, others from the store; best effort)."""
        now = time.time()
        out = {self.rank: current()}
        for r in range(self.world):
            if r == self.rank:
                continue
            raw = self._get(_PROG.format(r)) if self.store is not None else None
            out[r] = json.loads(raw) if raw else {"phase": "unknown (no progress record)", "t": None, "rank": r}
        for s in out.values():
            s["stalled_s"] = None if s.get("t") is None else round(now - s["t"], 1)
        return dict(sorted(out.items()))

    def _errors(self) -> List[Dict]:
        if self.store is None:
            return []
        try:
            n = self.store.add(_ERR_COUNT, 0)
        except Exception:  # noqa: BLE001
            return []
        if n <= 0:
            return []
        errs = []
        for r in range(self.world):
            raw = self._get(_ERR_KEY.format(r))
            if raw:
                errs.append(json.loads(raw))
        return errs

    # ------------------------------------------------------------------ failure paths
    def report_error(self, message: str) -> None:
        """Called by a rank whose main loop raised: record the error where rank 0 can see it and
        wait (bounded) for rank 0's failure line before this process exits."""
        rec = {"rank": self.rank, "phase": current()["phase"], "error": message[-2000:]}
        self._publish(current())
        if self.rank == 0 or self.store is None:
            self._fire("error", [rec])
            return
        try:
            self.store.set(_ERR_KEY.format(self.rank), json.dumps(rec))
            self.store.add(_ERR_COUNT, 1)
            self.store.wait([_ACK], datetime.timedelta(seconds=self.grace_s))
        except Exception:  # noqa: BLE001 - no acknowledgement: exit anyway
            pass

    def _fire(self, kind: str, errors: List[Dict]) -> None:
        if not self._fired.acquire(blocking=False):
            return
        try:
            if self.on_failure is not None:
                self.on_failure(kind, self.snapshot(), errors)
            if self.store is not None:
                try:
                    self.store.set(_ACK, "1")
                except Exception:  # noqa: BLE001
                    pass
            sys.stdout.flush()
            sys.stderr.flush()
        finally:
            os._exit(self.exit_code)

    def _stale_rank(self) -> Optional[int]:
        """(rank 0) a rank whose published mark is older than ``stall_s`` (None: all advancing)."""
        now = time.time()
        for r in range(self.world):
            st = current() if r == self.rank else None
            if st is None:
                raw = self._get(_PROG.format(r))
                if not raw:
                    continue
                st = json.loads(raw)
            if st.get("done"):
                continue
            if now - st["t"] > self.stall_s:
                return r
        return None

    def finish(self) -> None:
        """Mark this rank done (no stall reports after the timed loop) and stop the thread."""
        with _lock:
            _state["done"] = True
        self._publish(current())
        self.stop()

    def _run(self) -> None:
        while not self._stop.wait(self.publish_s):
            st = current()
            self._publish(st)
            if st.get("done"):
                continue
            if self.rank == 0:
                errs = self._errors()
                if errs:
                    self._fire("error", errs)
                if self.stall_s > 0 and self._stale_rank() is not None:
                    self._fire("stall", [])
            elif self.stall_s > 0 and time.time() - st["t"] > self.stall_s + self.grace_s:
                # rank 0 did not report (it may be the one that is gone): leave on our own
                print(f"[tdl] rank {self.rank} stalled {time.time() - st['t']:.0f}s in '{st['phase']}'",
                      file=sys.stderr, flush=True)
                os._exit(self.exit_code)
