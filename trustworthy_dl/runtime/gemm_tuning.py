"""hipBLASLt solution selection for the plain library GEMMs (PyTorch TunableOp, lookup only).

The GPT-2 step keeps its plain projections (qkv / out / proj forward, qkv / out / fc input
gradients, the LM head's logits and dX) on the library GEMM (ops/block.py: the native kernel
reaches 0.83-0.93x of it there).  hipBLASLt picks a solution per shape by heuristic; TunableOp
times every candidate solution of a shape once (scripts/gpu_r3_tunableop.sh on an MI355X) and
stores the winners in a CSV.  This module enables TunableOp in lookup-only mode with that file:
shapes in the file run their measured-fastest solution, every other shape the default heuristic;
nothing is tuned at run time.  The file records the torch / ROCm / hipBLASLt versions and the
gfx arch it was measured on; TunableOp refuses a file from a different stack.

    TDL_TUNED_GEMMS=0            disable
    TDL_TUNED_GEMMS=<path.csv>   use another results file
"""
from __future__ import annotations

import logging
import os
from typing import Optional

logger = logging.getLogger(__name__)

_DEFAULT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning",
                        "tunableop_gpt2m_mi355x.csv")
_state = {"done": False, "path": None}


def enable_tuned_gemms(path: Optional[str] = None) -> Optional[str]:
    """Turn on lookup-only TunableOp with the committed results file (idempotent).  Returns the
    file in use, or None (no file, disabled, no GPU, or TunableOp unavailable)."""
    if _state["done"]:
        return _state["path"]
    _state["done"] = True
    want = os.environ.get("TDL_TUNED_GEMMS", "1")
    if want == "0":
        return None
    path = path or (want if want not in ("1", "") else _DEFAULT)
    if not os.path.exists(path):
        return None
    try:
        import torch
        if not torch.cuda.is_available():
            return None
        from torch.cuda import tunable
        if os.environ.get("PYTORCH_TUNABLEOP_ENABLED") is not None:
            return None   # the caller drives TunableOp itself (tuning runs, A/B)
        import tempfile
        tunable.enable(True)
        tunable.tuning_enable(False)
        # whatever TunableOp writes back at exit goes to a scratch file, never over the committed one
        tunable.set_filename(os.path.join(tempfile.gettempdir(), f"tdl_tunableop_{os.getpid()}.csv"))
        if not tunable.read_file(path):
            raise RuntimeError("TunableOp rejected the file")
    except Exception as e:  # noqa: BLE001 - optional speed-up: never fatal
        logger.warning("tuned GEMM file %s not used: %s", path, e)
        try:
            from torch.cuda import tunable
            tunable.enable(False)
        except Exception:  # noqa: BLE001
            pass
        return None
    _state["path"] = path
    return path
