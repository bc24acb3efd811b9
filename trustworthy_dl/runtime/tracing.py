"""Per-phase step tracing with HIP events ("Tracing / profiling").

The reference only stamps ``time.time()`` into its attack and reassignment records
(distributed_trainer.py:280, 307, 347) and times whole epochs (experiment_runner.py:117-170).  Here
every phase of a pipeline step is bracketed by a pair of HIP events recorded on the compute
stream — forward, input-gradient backward, weight-gradient backward, the stall waiting for a
pipeline receive, verification (statistics + digest all-gather + trust update) and the optimizer
— so the breakdown is GPU time, measured without a host synchronisation.  Events are resolved
lazily (``resolve``) once the step's last event has completed, a step or two later, so tracing
does not stall the device queue.  On CPU (gloo tests) execution is synchronous and host clocks
are used instead.

    tr = PhaseTracer(device, enabled=True)
    with tr.phase("fwd"): ...
    tr.end_step(step)
    tr.resolve(); tr.summary()            # {"fwd": ms/step, ...}
    tr.export_chrome_trace("trace.json")  # chrome://tracing / Perfetto
"""
from __future__ import annotations

import contextlib
import json
import time
from collections import defaultdict, deque
from typing import Deque, Dict, List, Optional, Tuple

import torch

PHASES = ("fwd", "bwd_input", "bwd_weight", "p2p_wait", "verify", "optimizer")

_NULL = contextlib.nullcontext()


class _Span:
    __slots__ = ("tracer", "name", "start")

    def __init__(self, tracer: "PhaseTracer", name: str):
        self.tracer, self.name, self.start = tracer, name, None

    def __enter__(self):
        self.start = self.tracer._stamp()
        return self

    def __exit__(self, *exc):
        self.tracer._open.append((self.name, self.start, self.tracer._stamp()))
        return False


class PhaseTracer:
    def __init__(self, device: torch.device, enabled: bool = False, keep: int = 256):
        self.device = torch.device(device)
        self.enabled = enabled
        self.gpu = self.device.type == "cuda"
        self._open: List[Tuple[str, object, object]] = []
        self._origin = None
        self._pending: Deque[Tuple[int, object, List[Tuple[str, object, object]]]] = deque()
        self.steps: Deque[Tuple[int, Dict[str, float]]] = deque(maxlen=keep)
        self.spans: Deque[Tuple[int, str, float, float]] = deque(maxlen=keep * 64)

    # ---------------------------------------------------------------- recording
    def _stamp(self):
        if self.gpu:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(torch.cuda.current_stream(self.device))
            return ev
        return time.perf_counter()

    def phase(self, name: str):
        """Context manager bracketing one phase (a no-op when tracing is off)."""
        if not self.enabled:
            return _NULL
        if self._origin is None:
            self._origin = self._stamp()
        return _Span(self, name)

    def begin(self, name: str):
        """Open a phase without a ``with`` block; pass the token to ``end``."""
        if not self.enabled:
            return None
        sp = self.phase(name)
        sp.__enter__()
        return sp

    def end(self, token) -> None:
        if token is not None:
            token.__exit__(None, None, None)

    def wrap(self, name: str, fn):
        """``fn`` with every call bracketed as phase ``name`` (``fn`` itself when tracing is off)."""
        if not self.enabled:
            return fn

        def traced(*a, **k):
            with self.phase(name):
                return fn(*a, **k)
        return traced

    def end_step(self, step: int) -> None:
        if not self.enabled or self._origin is None:
            return
        self._pending.append((step, self._origin, self._open))
        self._open, self._origin = [], None
        if len(self._pending) > 16:        # never let an unread backlog grow without bound
            self.resolve(block=True)

    # ---------------------------------------------------------------- resolution
    def _elapsed_ms(self, a, b) -> float:
        return a.elapsed_time(b) if self.gpu else (b - a) * 1e3

    def resolve(self, block: bool = False) -> int:
        """Turn completed steps' events into per-phase times; returns how many steps resolved."""
        n = 0
        while self._pending:
            step, origin, spans = self._pending[0]
            if self.gpu and spans:
                last = spans[-1][2]
                if not last.query():
                    if not block:
                        break
                    last.synchronize()
            self._pending.popleft()
            acc: Dict[str, float] = defaultdict(float)
            for name, a, b in spans:
                ms = self._elapsed_ms(a, b)
                acc[name] += ms
                self.spans.append((step, name, self._elapsed_ms(origin, a), ms))
            if spans:
                acc["step"] = self._elapsed_ms(origin, spans[-1][2])
            self.steps.append((step, dict(acc)))
            n += 1
        return n

    # ---------------------------------------------------------------- reporting
    def last(self) -> Optional[Dict[str, float]]:
        return self.steps[-1][1] if self.steps else None

    def summary(self, skip: int = 0) -> Dict[str, float]:
        """Mean milliseconds per step of every phase over the resolved steps (after ``skip``)."""
        rows = [r for _, r in list(self.steps)[skip:]]
        if not rows:
            return {}
        keys = sorted({k for r in rows for k in r})
        return {k: sum(r.get(k, 0.0) for r in rows) / len(rows) for k in keys}

    def export_chrome_trace(self, path: str, pid: int = 0) -> None:
        """Chrome trace-event JSON ("X" events, microseconds relative to each step's first phase;
        steps are laid end to end on the timeline)."""
        events, base, cur = [], 0.0, None
        step_len: Dict[int, float] = {s: r.get("step", 0.0) for s, r in self.steps}
        for step, name, start_ms, dur_ms in self.spans:
            if step != cur:
                if cur is not None:
                    base += step_len.get(cur, 0.0) * 1e3
                cur = step
            events.append({"name": name, "ph": "X", "pid": pid, "tid": 0, "ts": base + start_ms * 1e3,
                           "dur": dur_ms * 1e3, "args": {"step": step}})
        with open(path, "w") as f:
            json.dump({"traceEvents": events, "displayTimeUnit": "ms"}, f)
