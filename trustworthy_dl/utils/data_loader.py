"""``get_dataloader(name, split, batch_size)`` (experiment_runner.py:100-110; phantom in the reference).

Datasets: ``openwebtext`` (README.md:80) / any ``*text*`` name -> token streams for language
modelling; ``cifar10`` (README.md:102) -> 3x32x32 images, 10 classes; ``imagenet`` ->
3x224x224 images, 1000 classes.  There is no network access in this environment, so every
loader yields *synthetic* data of the right shape (documented in the batch's ``"synthetic"``
flag): deterministic per (seed, split, index).  A local directory of ``.npy`` token shards or
a torchvision-style CIFAR folder can be plugged in through ``data_dir``.
Batches are dicts ``{"input": Tensor, "target": Tensor}`` (distributed_trainer.py:395, 398).

``native=True`` (language modelling) switches to the C++ loader (runtime/native.py,
csrc/runtime/token_loader.cpp): worker threads fill a pinned ring from a memory-mapped raw token
file (``token_file``, uint16/uint32) or synthetic ids, ahead of the training loop.
"""
from __future__ import annotations

import glob
import os
from typing import Dict, Iterator, Optional

import numpy as np
import torch


class SyntheticLanguageModeling:
    """Random token windows; target = input shifted by one (next-token prediction)."""

    def __init__(self, batch_size: int, seq_len: int = 1024, vocab_size: int = 50257, num_batches: int = 100,
                 seed: int = 0, split: str = "train", data_dir: Optional[str] = None, pin_memory: bool = False):
        self.batch_size, self.seq_len, self.vocab_size = batch_size, seq_len, vocab_size
        self.num_batches = num_batches
        self.seed = seed + (0 if split == "train" else 10_000)
        self.pin = pin_memory and torch.cuda.is_available()
        self.tokens = None
        if data_dir:
            shards = sorted(glob.glob(os.path.join(data_dir, "*.npy")))
            if shards:
                self.tokens = np.concatenate([np.load(s, allow_pickle=False).astype(np.int64) for s in shards])

    def __len__(self):
        return self.num_batches

    def __iter__(self) -> Iterator[Dict[str, torch.Tensor]]:
        for i in range(self.num_batches):
            g = torch.Generator().manual_seed(self.seed * 100_003 + i)
            if self.tokens is not None:
                starts = torch.randint(0, len(self.tokens) - self.seq_len - 1, (self.batch_size,), generator=g)
                ids = torch.stack([torch.from_numpy(self.tokens[s:s + self.seq_len + 1]) for s in starts.tolist()])
            else:
                ids = torch.randint(0, self.vocab_size, (self.batch_size, self.seq_len + 1), generator=g)
            b = {"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()}
            if self.pin:
                b = {k: v.pin_memory() for k, v in b.items()}
            yield b


class SyntheticImages:
    """Class-conditional Gaussian images (learnable signal, so loss decreases)."""

    def __init__(self, batch_size: int, image_size: int = 32, num_classes: int = 10, num_batches: int = 100,
                 seed: int = 0, split: str = "train", pin_memory: bool = False):
        self.batch_size, self.image_size, self.num_classes = batch_size, image_size, num_classes
        self.num_batches = num_batches
        self.seed = seed + (0 if split == "train" else 10_000)
        g = torch.Generator().manual_seed(seed)
        self.prototypes = torch.randn(num_classes, 3, 8, 8, generator=g)
        self.pin = pin_memory and torch.cuda.is_available()

    def __len__(self):
        return self.num_batches

    def __iter__(self):
        for i in range(self.num_batches):
            g = torch.Generator().manual_seed(self.seed * 100_003 + i)
            y = torch.randint(0, self.num_classes, (self.batch_size,), generator=g)
            base = torch.nn.functional.interpolate(self.prototypes[y], size=self.image_size, mode="nearest")
            x = base + 0.5 * torch.randn(self.batch_size, 3, self.image_size, self.image_size, generator=g)
            b = {"input": x, "target": y}
            if self.pin:
                b = {k: v.pin_memory() for k, v in b.items()}
            yield b


def get_dataloader(dataset_name: str, split: str = "train", batch_size: int = 32, seq_len: int = 1024,
                   num_batches: Optional[int] = None, seed: int = 0, data_dir: Optional[str] = None,
                   vocab_size: int = 50257, pin_memory: bool = False, native: bool = False,
                   token_file: Optional[str] = None, token_bytes: int = 2, rank: int = 0, world: int = 1):
    name = dataset_name.lower()
    nb = num_batches if num_batches is not None else (100 if split == "train" else 10)
    if "text" in name or name in ("openwebtext", "wikitext", "tokens", "lm"):
        if native or token_file:
            from ..runtime.native import NativeTokenLoader
            return NativeTokenLoader(batch_size, seq_len, path=token_file, vocab_size=vocab_size,
                                     token_bytes=token_bytes, seed=seed + (0 if split == "train" else 10_000),
                                     num_batches=nb, rank=rank, world=world, pin_memory=pin_memory or None)
        return SyntheticLanguageModeling(batch_size, seq_len, vocab_size, nb, seed, split, data_dir, pin_memory)
    if name in ("cifar10", "cifar-10", "cifar"):
        return SyntheticImages(batch_size, 32, 10, nb, seed, split, pin_memory)
    if name in ("cifar100", "cifar-100"):
        return SyntheticImages(batch_size, 32, 100, nb, seed, split, pin_memory)
    if name in ("imagenet", "imagenet1k", "imagenet-1k"):
        return SyntheticImages(batch_size, 224, 1000, nb, seed, split, pin_memory)
    raise ValueError(f"unknown dataset {dataset_name!r}")
