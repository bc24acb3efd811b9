import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# the engine draws the monitored micro-batch from a private RNG seeded from os.urandom in
# production (an attacker must not predict it); tests pin it so outcomes do not depend on the draw
os.environ.setdefault("TDL_MONITOR_SEED", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)
