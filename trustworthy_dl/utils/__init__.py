"""Utilities: metrics, data loaders, checkpointing."""
from .metrics import MetricsCollector  # noqa: F401
from .data_loader import get_dataloader  # noqa: F401
