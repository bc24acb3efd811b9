"""Data loaders: learnable Markov tokens, real image data from CIFAR binary batches / .npy arrays."""
import os

import numpy as np
import pytest
import torch

from trustworthy_dl.utils.data_loader import ImageArrays, get_dataloader


def test_cifar10_binary_batches(tmp_path):
    rng = np.random.default_rng(0)
    for i in range(1, 3):
        labels = rng.integers(0, 10, 50, dtype=np.uint8)
        pix = rng.integers(0, 256, (50, 3072), dtype=np.uint8)
        np.concatenate([labels[:, None], pix], 1).tofile(tmp_path / f"data_batch_{i}.bin")
    dl = get_dataloader("cifar10", "train", batch_size=16, data_dir=str(tmp_path))
    assert isinstance(dl, ImageArrays) and len(dl) == 100 // 16
    b = next(iter(dl))
    assert b["input"].shape == (16, 3, 32, 32) and b["input"].dtype == torch.float32
    assert b["target"].dtype == torch.int64 and int(b["target"].max()) < 10
    assert abs(float(b["input"].mean())) < 1.0


def test_npy_image_arrays(tmp_path):
    x = np.random.default_rng(1).integers(0, 256, (40, 32, 32, 3), dtype=np.uint8)   # NHWC
    np.save(tmp_path / "test_images.npy", x)
    np.save(tmp_path / "test_labels.npy", np.arange(40) % 10)
    dl = get_dataloader("cifar10", "test", batch_size=8, data_dir=str(tmp_path))
    batches = list(dl)
    assert len(batches) == 5 and batches[0]["input"].shape == (8, 3, 32, 32)
    assert sorted(torch.cat([b["target"] for b in batches]).tolist()) == sorted((np.arange(40) % 10).tolist())


def test_missing_image_dir_raises(tmp_path):
    with pytest.raises(FileNotFoundError):
        get_dataloader("cifar10", "train", batch_size=8, data_dir=str(tmp_path))


def test_markov_stream_via_factory():
    dl = get_dataloader("markov", "train", batch_size=2, seq_len=16, num_batches=2, vocab_size=128)
    b = next(iter(dl))
    assert b["input"].shape == (2, 16) and int(b["input"].max()) < 128
