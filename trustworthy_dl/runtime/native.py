"""ctypes bindings of the host C++ runtime (``trustworthy_dl/_native/libtdl_runtime.so``, csrc/runtime/).

Built in-tree by ``build_native.py`` (g++ -O2 -pthread); loaded once; raises if missing.
"""
from __future__ import annotations

import ctypes
import os
import threading
from collections import deque
from typing import Dict, Iterator, Optional

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.path.join(_HERE, "..", "_native", "libtdl_runtime.so"))
_lib: Optional[ctypes.CDLL] = None
_lock = threading.Lock()


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError(f"{LIB_PATH} not found: run `python build_native.py`")
                L = ctypes.CDLL(LIB_PATH)
                P, I, L64, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint64
                L.tdl_loader_create.argtypes = [ctypes.c_char_p, I, L64, I, I, U64, I, I, I, I]
                L.tdl_loader_create.restype = P
                L.tdl_loader_bind_slot.argtypes = [P, I, P, P]
                L.tdl_loader_bind_slot.restype = I
                L.tdl_loader_start.argtypes = [P]
                L.tdl_loader_start.restype = I
                L.tdl_loader_next.argtypes = [P, ctypes.POINTER(L64)]
                L.tdl_loader_next.restype = I
                L.tdl_loader_release.argtypes = [P, I]
                L.tdl_loader_release.restype = I
                L.tdl_loader_num_tokens.argtypes = [P]
                L.tdl_loader_num_tokens.restype = L64
                L.tdl_loader_destroy.argtypes = [P]
                L.tdl_loader_destroy.restype = None
                L.tdl_host_merkle.argtypes = [P, L64, I, P, P, I, I, P]
                L.tdl_host_merkle.restype = I
                _lib = L
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except (RuntimeError, OSError):
        return False


class NativeTokenLoader:
    """Iterable of ``{"input": [B, T], "target": [B, T]}`` int64 batches filled by C++ worker threads
    into a ring of (pinned, on GPU hosts) buffers.

    ``path``: raw little-endian token file (uint16 by default, ``token_bytes=4`` for uint32), read
    through mmap; ``None`` -> synthetic ids.  Batch k is a pure function of (seed, rank, k).
    A yielded batch's slot is handed back to the workers only after the consumer's stream has
    passed an event recorded at the following ``next()`` (its H2D copies are complete), so the
    non-blocking copies the engine issues never race a refill.
    """

    def __init__(self, batch_size: int, seq_len: int, path: Optional[str] = None, vocab_size: int = 50257,
                 token_bytes: int = 2, seed: int = 0, num_batches: Optional[int] = None, slots: int = 4,
                 threads: int = 2, rank: int = 0, world: int = 1, pin_memory: Optional[bool] = None):
        self.B, self.T = batch_size, seq_len
        self.num_batches = num_batches
        pin = torch.cuda.is_available() if pin_memory is None else pin_memory
        self._h = lib().tdl_loader_create(path.encode() if path else None, token_bytes, vocab_size, batch_size,
                                          seq_len, seed, slots, threads, rank, world)
        if not self._h:
            raise RuntimeError(f"tdl_loader_create failed (path={path!r}, token_bytes={token_bytes})")
        self._bufs = []
        for s in range(slots):
            inp = torch.empty(batch_size, seq_len, dtype=torch.int64, pin_memory=pin)
            tgt = torch.empty(batch_size, seq_len, dtype=torch.int64, pin_memory=pin)
            self._bufs.append((inp, tgt))
            if lib().tdl_loader_bind_slot(self._h, s, inp.data_ptr(), tgt.data_ptr()) != 0:
                raise RuntimeError("tdl_loader_bind_slot failed")
        if lib().tdl_loader_start(self._h) != 0:
            raise RuntimeError("tdl_loader_start failed")
        self._outstanding: deque = deque()
        self._max_out = max(1, slots - 2)
        self.produced = 0

    @property
    def num_tokens(self) -> int:
        return int(lib().tdl_loader_num_tokens(self._h))

    def _retire(self, block: bool):
        while self._outstanding:
            slot, ev = self._outstanding[0]
            if ev is not None and not ev.query():
                if not (block or len(self._outstanding) > self._max_out):
                    return
                ev.synchronize()
            self._outstanding.popleft()
            lib().tdl_loader_release(self._h, slot)

    def next_batch(self) -> Dict[str, torch.Tensor]:
        # the previous batch's consumers have enqueued their copies by now: fence them
        if self._outstanding and self._outstanding[-1][1] is None and torch.cuda.is_available():
            slot, _ = self._outstanding.pop()
            ev = torch.cuda.Event()
            ev.record()
            self._outstanding.append((slot, ev))
        self._retire(block=False)
        k = ctypes.c_int64(-1)
        slot = lib().tdl_loader_next(self._h, ctypes.byref(k))
        if slot < 0:
            raise RuntimeError("native loader stopped")
        self._outstanding.append((slot, None))
        if not torch.cuda.is_available():
            # host consumer: the batch is used synchronously before the next call
            pass
        inp, tgt = self._bufs[slot]
        self.produced += 1
        return {"input": inp, "target": tgt, "batch_index": int(k.value)}

    def __len__(self):
        return self.num_batches if self.num_batches is not None else 0

    def __iter__(self) -> Iterator[Dict[str, torch.Tensor]]:
        n = 0
        while self.num_batches is None or n < self.num_batches:
            b = self.next_batch()
            yield {"input": b["input"], "target": b["target"]}
            n += 1

    def close(self):
        if getattr(self, "_h", None):
            self._outstanding.clear()
            lib().tdl_loader_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
