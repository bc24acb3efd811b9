"""Hardware-queue budget for the HIP runtime (``GPU_MAX_HW_QUEUES``).

HIP maps every stream onto one of ``GPU_MAX_HW_QUEUES`` hardware queues (4 by default); streams
beyond that share a queue, and a kernel on one stream then waits behind every earlier kernel of
the other streams on that queue.  ``scripts/hwqueue_probe.py`` measures it on MI355X
(profiles/r1_hwqueue_probe.json): with 4 queues the null stream shares its queue with two of
twelve pool streams, and a kernel on either waits for a spinning kernel on the other; with 16
queues none of the 13 streams share.

The pipeline posts RCCL receives a compute phase ahead (parallel/pipeline.py, ``p2p_mode="async"``)
on per-neighbour communicator streams.  An RCCL receive kernel spins until the peer's data lands, so
if its stream shares a queue with the compute stream, the stage's compute stalls behind it; when
two neighbouring stages both pre-post receives the peer can only satisfy after that compute, the
two GPUs wait on each other.  A pipeline stage uses about 12 streams (compute, verification side
stream, default/activation/gradient/tie communicators and their per-neighbour P2P streams), so
the engine asks for 32 queues (the most this pool's boxes allow; queues are created only as
streams are, so unused headroom costs nothing) and keeps pre-posted receives only with >= 16.

The variable is read once, when the HIP runtime initialises, so :func:`ensure_hw_queues` must run
before the first GPU call; importing ``trustworthy_dl`` does it.  ``TDL_KEEP_HW_QUEUES=1`` leaves
the environment alone.
"""
from __future__ import annotations

import os
import sys

HIP_DEFAULT_QUEUES = 4
REQUEST_QUEUES = 32     # asked for before the HIP runtime starts
ENGINE_QUEUES = 16      # fewer than this: the pipeline does not pre-post receives
_effective = None   # queue count the HIP runtime of this process started (or will start) with


def _hip_initialized() -> bool:
    torch = sys.modules.get("torch")
    if torch is None:
        return False
    try:
        return bool(torch.cuda.is_initialized())
    except Exception:
        return False


def _env_queues() -> int:
    try:
        return int(os.environ.get("GPU_MAX_HW_QUEUES", HIP_DEFAULT_QUEUES))
    except ValueError:
        return HIP_DEFAULT_QUEUES


def ensure_hw_queues(min_queues: int = REQUEST_QUEUES) -> int:
    """Raise ``GPU_MAX_HW_QUEUES`` to ``min_queues`` if the HIP runtime has not started yet.
    Returns the queue count this process runs (or will run) with."""
    global _effective
    if _effective is not None:
        return _effective
    cur = _env_queues()
    if _hip_initialized():
        _effective = cur                      # too late to change: report what HIP started with
    elif cur < min_queues and os.environ.get("TDL_KEEP_HW_QUEUES", "0") != "1":
        os.environ["GPU_MAX_HW_QUEUES"] = str(min_queues)
        _effective = min_queues
    else:
        _effective = cur
    return _effective


def effective_hw_queues() -> int:
    """Queue count of this process's HIP runtime (as far as this module could see or set it)."""
    return _effective if _effective is not None else _env_queues()


def _reset_for_tests():
    global _effective
    _effective = None
