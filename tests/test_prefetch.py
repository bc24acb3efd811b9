"""utils/prefetch.DevicePrefetcher: one batch ahead on a copy stream, values intact, only the
requested entries moved (CPU: pass-through)."""
import pytest
import torch

from trustworthy_dl.utils.prefetch import DevicePrefetcher


def _batches(n, dev_pin=False):
    out = []
    for i in range(n):
        x = torch.full((4, 8), float(i))
        y = torch.arange(4) + i
        if dev_pin:
            x, y = x.pin_memory(), y.pin_memory()
        out.append({"input": x, "target": y, "meta": i})
    return out


def test_cpu_pass_through():
    src = _batches(3)
    got = list(DevicePrefetcher(iter(src), "cpu"))
    assert len(got) == 3
    for i, b in enumerate(got):
        assert b["meta"] == i and torch.equal(b["input"], src[i]["input"])


@pytest.mark.gpu
def test_gpu_copies_ahead_and_filters_keys():
    src = _batches(4, dev_pin=True)
    pf = DevicePrefetcher(iter(src), "cuda", keys=["input"])
    for i in range(4):
        b = next(pf)
        assert b["input"].is_cuda and not b["target"].is_cuda
        # consume on the compute stream right away: the event wait must order it after the copy
        assert float(b["input"].sum()) == 32.0 * i
        assert torch.equal(b["target"], src[i]["target"])
    with pytest.raises(StopIteration):
        next(pf)
