"""Host -> device batch prefetch on a side HIP stream.

The engine moves each step's batch to its device with ``non_blocking`` copies on the compute stream,
so the copy of a ResNet-50 batch (64 x 3 x 224 x 224 fp32, 38.5 MB) sat in front of the first
convolution: ~0.7 ms of a 13.5 ms step (profiles/r5_copy_probe_resnet50.txt).  ``DevicePrefetcher``
issues the NEXT batch's copies on a copy stream as soon as the current batch is handed out, so they
run under the current step's compute; the compute stream waits on an event before it touches the
batch, and the tensors are recorded on it so the caching allocator does not recycle them early.

Reference: the training loop hands each dataloader batch straight to the forward pass
(/root/reference/distributed_trainer.py:391-398), with no prefetch.
"""
from __future__ import annotations

from typing import Dict, Iterable, Iterator, Optional, Sequence

import torch


class DevicePrefetcher:
    """Iterate ``batches`` (dicts of tensors, host memory — pinned for the copies to be asynchronous)
    as device batches, one batch ahead.  ``keys`` restricts the copies to the entries this rank
    consumes (e.g. only the first pipeline stage needs the images); the others are passed through
    on the host.  On a CPU device it is a plain pass-through."""

    def __init__(self, batches: Iterable[Dict[str, torch.Tensor]], device, keys: Optional[Sequence[str]] = None):
        self.it: Iterator = iter(batches)
        self.device = torch.device(device)
        self.keys = None if keys is None else set(keys)
        self.cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(self.device) if self.cuda else None
        self._next: Optional[Dict[str, torch.Tensor]] = None
        self._event = None
        self._load()

    def _moves(self, k: str, v) -> bool:
        return torch.is_tensor(v) and (self.keys is None or k in self.keys)

    def _load(self):
        try:
            b = next(self.it)
        except StopIteration:
            self._next = None
            return
        if not self.cuda:
            self._next = b
            return
        # the copy stream must not start before the compute stream is done with what it overwrites
        # (nothing: every batch gets fresh device memory), only after the host data exists
        with torch.cuda.stream(self.stream):
            self._next = {k: (v.to(self.device, non_blocking=True) if self._moves(k, v) else v) for k, v in b.items()}
            self._event = torch.cuda.Event()
            self._event.record(self.stream)

    def __iter__(self):
        return self

    def __next__(self) -> Dict[str, torch.Tensor]:
        if self._next is None:
            raise StopIteration
        b = self._next
        if self.cuda:
            cur = torch.cuda.current_stream(self.device)
            cur.wait_event(self._event)
            for k, v in b.items():
                if self._moves(k, v):
                    v.record_stream(cur)
        self._load()
        return b
