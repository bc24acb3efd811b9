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
