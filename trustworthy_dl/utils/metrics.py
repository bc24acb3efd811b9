"""``MetricsCollector`` — per-batch metric accumulation and summaries.

Imported by the reference trainer and runner (distributed_trainer.py:23, 83, 417, 520;
experiment_runner.py:25) with ``collect_batch_metrics(dict)`` and ``get_summary()`` but never
shipped.  Adds throughput, step-time percentiles, detection counts, JSONL/CSV export
and real device memory statistics (HIP allocator) instead of the reference's simulated
``np.random`` system metrics (experiment_runner.py:262-268).
"""
from __future__ import annotations

import csv
import json
import glob
import os
import time
from collections import defaultdict
from typing import Any, Dict, List, Optional

import numpy as np
import torch


class MetricsCollector:
    def __init__(self, tokens_per_step: Optional[int] = None, jsonl_path: Optional[str] = None):
        self.batch_metrics: List[Dict[str, Any]] = []
        self.epoch_metrics: List[Dict[str, Any]] = []
        self.counters = defaultdict(float)
        self.tokens_per_step = tokens_per_step
        self.jsonl_path = jsonl_path
        self._t0 = time.time()

    def collect_batch_metrics(self, metrics: Dict[str, Any]):
        m = dict(metrics)
        m.setdefault("timestamp", time.time())
        self.batch_metrics.append(m)
        if m.get("detections"):
            self.counters["detections"] += len(m["detections"])
        if self.jsonl_path:
            with open(self.jsonl_path, "a") as f:
                f.write(json.dumps(m, default=float) + "\n")

    def collect_epoch_metrics(self, metrics: Dict[str, Any]):
        self.epoch_metrics.append(dict(metrics))

    def increment(self, key: str, value: float = 1.0):
        self.counters[key] += value

    @staticmethod
    def device_memory() -> Dict[str, float]:
        if not torch.cuda.is_available():
            return {}
        free, total = torch.cuda.mem_get_info()
        return {"allocated_gb": torch.cuda.memory_allocated() / 2 ** 30,
                "reserved_gb": torch.cuda.memory_reserved() / 2 ** 30,
                "max_allocated_gb": torch.cuda.max_memory_allocated() / 2 ** 30,
                "hbm_used_fraction": 1.0 - free / total}

    @staticmethod
    def gpu_system_metrics(device_index: Optional[int] = None) -> Dict[str, float]:
        """Measured device counters from the amdgpu driver's sysfs (what rocm-smi / amd-smi read):
        ``gpu_busy_percent``, ``mem_busy_percent``, socket power (W) and edge/junction temperature
        (C) of the card hosting ``device_index`` (matched by PCI address).  Empty when no AMD GPU is
        visible (CPU runs).  The reference simulates these (experiment_runner.py:262-274)."""
        if not torch.cuda.is_available():
            return {}
        idx = torch.cuda.current_device() if device_index is None else device_index
        card = _drm_card_for(idx)
        if card is None:
            return {}
        out: Dict[str, float] = {}
        for key, fname in (("gpu_busy_percent", "gpu_busy_percent"), ("mem_busy_percent", "mem_busy_percent")):
            v = _read_num(os.path.join(card, fname))
            if v is not None:
                out[key] = v
        for hw in glob.glob(os.path.join(card, "hwmon", "hwmon*")):
            for key, fname, scale in (("power_w", "power1_average", 1e-6), ("power_w", "power1_input", 1e-6),
                                      ("temp_edge_c", "temp1_input", 1e-3), ("temp_junction_c", "temp2_input", 1e-3),
                                      ("temp_mem_c", "temp3_input", 1e-3)):
                v = _read_num(os.path.join(hw, fname))
                if v is not None and key not in out:
                    out[key] = v * scale
        return out

    def get_summary(self) -> Dict[str, Any]:
        losses = [m["loss"] for m in self.batch_metrics if m.get("loss") is not None]
        times = [m["step_time"] for m in self.batch_metrics if m.get("step_time")]
        out: Dict[str, Any] = {"num_batches": len(self.batch_metrics), "wall_time_s": time.time() - self._t0}
        if losses:
            out.update({"mean_loss": float(np.mean(losses)), "final_loss": float(losses[-1]),
                        "min_loss": float(np.min(losses)), "initial_loss": float(losses[0])})
        if times:
            out.update({"mean_step_time_s": float(np.mean(times)), "p50_step_time_s": float(np.percentile(times, 50)),
                        "p95_step_time_s": float(np.percentile(times, 95))})
            if self.tokens_per_step:
                out["tokens_per_s"] = self.tokens_per_step / float(np.mean(times))
        out.update({k: v for k, v in self.counters.items()})
        return out

    def to_csv(self, path: str, keys=("step", "epoch", "loss", "timestamp")):
        with open(path, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(keys)
            for m in self.batch_metrics:
                w.writerow([m.get(k) for k in keys])

    def reset(self):
        self.batch_metrics.clear()
        self.epoch_metrics.clear()
        self.counters.clear()


def _read_num(path: str) -> Optional[float]:
    try:
        with open(path) as f:
            return float(f.read().strip().split()[0])
    except (OSError, ValueError, IndexError):
        return None


_CARD_CACHE: Dict[int, Optional[str]] = {}


def _drm_card_for(device_index: int) -> Optional[str]:
    """sysfs device directory of the DRM card whose PCI address matches the HIP device."""
    if device_index in _CARD_CACHE:
        return _CARD_CACHE[device_index]
    found = None
    try:
        pr = torch.cuda.get_device_properties(device_index)
        want = (int(getattr(pr, "pci_domain_id", 0)), int(pr.pci_bus_id), int(getattr(pr, "pci_device_id", 0)))
    except Exception:  # noqa: BLE001
        want = None
    cards = sorted(glob.glob("/sys/class/drm/card[0-9]*/device"))
    for dev in cards:
        if not os.path.exists(os.path.join(dev, "gpu_busy_percent")):
            continue
        addr = os.path.basename(os.path.realpath(dev))          # e.g. 0000:75:00.0
        try:
            dom, bus, rest = addr.split(":")
            slot = int(rest.split(".")[0], 16)
            key = (int(dom, 16), int(bus, 16), slot)
        except ValueError:
            continue
        if want is not None and key == want:
            found = dev
            break
    if found is None and want is None and cards:
        found = cards[0]
    _CARD_CACHE[device_index] = found
    return found
