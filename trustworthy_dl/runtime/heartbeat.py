"""Heartbeat watchdog: the source of ``NodeStatus.OFFLINE`` (trust_manager.py:23 in the reference
defines the state but nothing ever sets it — SURVEY §5 "Crash/OFFLINE").

Every rank runs one daemon thread that, each ``interval`` seconds, bumps its own counter in the
process group's c10d store (``store.add("tdl/hb/<rank>", 1)``: atomic, non-blocking, works for
RCCL and gloo groups alike) and reads every peer's counter (``add(key, 0)``).  A peer whose
counter has not advanced for ``timeout`` seconds is reported offline; when it advances again it
is reported back online.  The watchdog is deliberately outside the GPU/RCCL path: a rank whose
training loop is stuck inside a collective still beats (its process is alive), while a crashed
or hung process stops — which is exactly the distinction between a slow peer and a dead one.
``abort_on_offline`` turns detection into fail-fast (``os._exit``), so an elastic launcher
(torchrun --max-restarts) restarts the job from the latest checkpoint instead of hanging in RCCL.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from typing import Callable, Dict, Optional, Set

logger = logging.getLogger(__name__)


class HeartbeatMonitor:
    def __init__(self, store, rank: int, world: int, interval: float = 1.0, timeout: float = 30.0,
                 on_offline: Optional[Callable[[int], None]] = None,
                 on_online: Optional[Callable[[int], None]] = None,
                 abort_on_offline: bool = False, prefix: str = "tdl/hb"):
        self.store, self.rank, self.world = store, rank, world
        self.interval, self.timeout = float(interval), float(timeout)
        self.on_offline, self.on_online = on_offline, on_online
        self.abort_on_offline = abort_on_offline
        self.prefix = prefix
        self._last_val: Dict[int, int] = {}
        self._last_change: Dict[int, float] = {}
        self._offline: Set[int] = set()
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._paused = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.events = []
        self._store_fail_since: Optional[float] = None  # first of the current run of store errors
        self.store_host = 0  # the rank hosting the c10d TCPStore (torch.distributed: rank 0)

    def _report_offline(self):
        """Tell the elastic supervisor (runtime/elastic.py) whom this rank saw go silent: the vote
        that separates the lost ranks from the ones that merely went down with them."""
        d = os.environ.get("TDL_ELASTIC_REPORT_DIR")
        if not d:
            return
        try:
            import json
            os.makedirs(d, exist_ok=True)
            with open(os.path.join(d, f"offline.rank{self.rank}.json"), "w") as f:
                json.dump(sorted(self._offline), f)
        except OSError as exc:
            logger.error("heartbeat: could not write the offline report: %s", exc)

    def _key(self, r: int) -> str:
        return f"{self.prefix}/{r}"

    def beat(self):
        self.store.add(self._key(self.rank), 1)

    def poll(self, now: Optional[float] = None):
        now = time.monotonic() if now is None else now
        for r in range(self.world):
            if r == self.rank:
                continue
            v = int(self.store.add(self._key(r), 0))
            with self._lock:
                if self._last_val.get(r) != v:
                    self._last_val[r] = v
                    self._last_change[r] = now
                    if r in self._offline:
                        self._offline.discard(r)
                        self.events.append({"node_id": r, "event": "online", "time": time.time()})
                        logger.warning("heartbeat: node %d is back online", r)
                        if self.on_online:
                            self.on_online(r)
                elif r not in self._offline and now - self._last_change.get(r, now) > self.timeout:
                    self._offline.add(r)
                    self.events.append({"node_id": r, "event": "offline", "time": time.time()})
                    logger.error("heartbeat: node %d silent for > %.1fs -> OFFLINE", r, self.timeout)
                    if self.on_offline:
                        self.on_offline(r)
                    if self.abort_on_offline:
                        logger.error("heartbeat: aborting (fail-fast) so the elastic launcher can restart")
                        self._report_offline()
                        os._exit(17)
                self._last_change.setdefault(r, now)

    def store_failed(self, exc: Exception, now: Optional[float] = None):
        """The store itself is unreachable.  It lives in the store host's process (rank 0), so when
        that rank dies every survivor's beat / poll fails: after ``timeout`` seconds of consecutive
        failures the host is declared OFFLINE like any silent peer (with ``abort_on_offline`` the
        survivors report it and exit 17 instead of sitting in RCCL until the supervisor's grace
        period runs out).  A single failure (store busy, shutdown) only starts the clock."""
        now = time.monotonic() if now is None else now
        if self._store_fail_since is None:
            self._store_fail_since = now
            logger.debug("heartbeat: store error (%s)", exc)
            return
        host = self.store_host
        if host == self.rank or now - self._store_fail_since <= self.timeout:
            return
        with self._lock:
            if host in self._offline:
                return
            self._offline.add(host)
            self.events.append({"node_id": host, "event": "offline", "time": time.time(), "reason": "store"})
        logger.error("heartbeat: store on rank %d unreachable for > %.1fs -> node %d OFFLINE (%s)", host,
                     self.timeout, host, exc)
        if self.on_offline:
            self.on_offline(host)
        if self.abort_on_offline:
            self._report_offline()
            os._exit(17)

    def _run(self):
        while not self._stop.is_set():
            if not self._paused.is_set():
                try:
                    self.beat()
                    self.poll()
                    self._store_fail_since = None
                except Exception as e:  # noqa: BLE001 - store gone (host died, or shutdown)
                    if not self._stop.is_set():
                        self.store_failed(e)
            self._stop.wait(self.interval)

    def start(self) -> "HeartbeatMonitor":
        self.beat()
        self._thread = threading.Thread(target=self._run, name="tdl-heartbeat", daemon=True)
        self._thread.start()
        return self

    def pause(self):
        """Stop beating (and polling): simulates a hung / dead process in tests."""
        self._paused.set()

    def resume(self):
        self._paused.clear()

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5 * self.interval + 1)

    def offline(self) -> Set[int]:
        with self._lock:
            return set(self._offline)
