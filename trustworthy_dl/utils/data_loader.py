"""``get_dataloader(name, split, batch_size)`` (experiment_runner.py:100-110; phantom in the reference).

Datasets: ``openwebtext`` (README.md:80) / any ``*text*`` name -> token streams for language
modelling; ``markov`` -> a learnable synthetic token stream (order-k Markov chain); ``cifar10`` (README.md:102) -> 3x32x32 images, 10 classes; ``imagenet`` ->
3x224x224 images, 1000 classes.  There is no network access in this environment, so every
loader yields *synthetic* data of the right shape (documented in the batch's ``"synthetic"``
flag): deterministic per (seed, split, index).  Real data plugs in through ``data_dir``: ``.npy``
token shards for language modelling, the CIFAR-10/100 binary release or ``{split}_images.npy`` +
``{split}_labels.npy`` arrays for images (``ImageArrays``; nothing is unpickled).
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


class MarkovLanguageModeling:
    """Learnable synthetic token stream: an order-``order`` Markov chain over the vocabulary.

    Each context (the previous ``order`` tokens) has ``branching`` successor tokens, picked by a
    fixed hash of the context and the chain's seed, with Zipf-like probabilities.  A language
    model can learn it — the loss falls from ln(V) towards the chain's entropy (about 1.2 nats for
    the default branching 4) — so gradients drift and correlate from step to step the way real
    training's do, unlike uniform random tokens whose loss and gradients stay flat.  Used to
    measure detection false-positive rates under learning (bench_detection.py --data markov).
    Deterministic per (seed, split, batch index)."""

    _PROBS = {2: [0.7, 0.3], 3: [0.6, 0.3, 0.1], 4: [0.6, 0.25, 0.1, 0.05]}

    def __init__(self, batch_size: int, seq_len: int = 1024, vocab_size: int = 50257, num_batches: int = 100,
                 seed: int = 0, split: str = "train", order: int = 1, branching: int = 4, pin_memory: bool = False):
        self.batch_size, self.seq_len, self.vocab_size = batch_size, seq_len, vocab_size
        self.num_batches = num_batches
        self.chain_seed = seed                      # the chain itself is the same for every split
        self.seed = seed + (0 if split == "train" else 10_000)
        self.order = max(1, int(order))
        probs = self._PROBS.get(branching) or list(np.full(branching, 1.0 / branching))
        self.cum = np.cumsum(np.asarray(probs, dtype=np.float64))
        self.cum[-1] = 1.0
        self.pin = pin_memory and torch.cuda.is_available()

    def entropy(self) -> float:
        p = np.diff(np.concatenate([[0.0], self.cum]))
        return float(-(p * np.log(p)).sum())

    def successor(self, ctx: np.ndarray, k: np.ndarray) -> np.ndarray:
        """Successor ``k`` of each context row (uint64 hash of the context tokens and the seed)."""
        h = np.full(ctx.shape[0], (self.chain_seed * 0x9E3779B97F4A7C15 + 0x632BE59BD9B4E019) & (2 ** 64 - 1),
                    dtype=np.uint64)
        with np.errstate(over="ignore"):
            for j in range(ctx.shape[1]):
                h = (h ^ ctx[:, j].astype(np.uint64)) * np.uint64(0x100000001B3)
                h ^= h >> np.uint64(29)
            h = (h + k.astype(np.uint64) * np.uint64(0xBF58476D1CE4E5B9)) * np.uint64(0x94D049BB133111EB)
            h ^= h >> np.uint64(31)
        return (h % np.uint64(self.vocab_size)).astype(np.int64)

    def __len__(self):
        return self.num_batches

    def __iter__(self):
        for i in range(self.num_batches):
            rng = np.random.default_rng(self.seed * 100_003 + i)
            B, T = self.batch_size, self.seq_len + 1
            ids = np.empty((B, T), dtype=np.int64)
            ids[:, :self.order] = rng.integers(0, self.vocab_size, (B, self.order))
            u = rng.random((B, T))
            for t in range(self.order, T):
                k = np.searchsorted(self.cum, u[:, t], side="right")
                ids[:, t] = self.successor(ids[:, t - self.order:t], k)
            ids = torch.from_numpy(ids)
            b = {"input": ids[:, :-1].contiguous(), "target": ids[:, 1:].contiguous()}
            if self.pin:
                b = {k_: v.pin_memory() for k_, v in b.items()}
            yield b


class ImageArrays:
    """Real image data from disk, no pickles:

    * the CIFAR-10/100 *binary* release (``data_batch_{1..5}.bin`` / ``test_batch.bin``, or
      ``train.bin`` / ``test.bin`` for CIFAR-100): records of label byte(s) + 3072 pixel bytes;
    * ``{split}_images.npy`` (uint8 [N, H, W, 3] or [N, 3, H, W]) + ``{split}_labels.npy``.

    Images are normalised per channel (CIFAR mean / std) and shuffled per epoch (seeded)."""

    _MEAN = np.array([0.4914, 0.4822, 0.4465], dtype=np.float32)
    _STD = np.array([0.2470, 0.2435, 0.2616], dtype=np.float32)

    def __init__(self, data_dir: str, batch_size: int, split: str = "train", num_batches: Optional[int] = None,
                 seed: int = 0, num_classes: int = 10, pin_memory: bool = False):
        self.batch_size, self.seed, self.num_classes = batch_size, seed, num_classes
        self.pin = pin_memory and torch.cuda.is_available()
        x, y = self._load(data_dir, split, num_classes)
        if x is None:
            raise FileNotFoundError(f"no CIFAR binary batches or {split}_images.npy in {data_dir}")
        self.x, self.y = x, y
        full = len(self.y) // batch_size
        self.num_batches = min(full, num_batches) if num_batches else full

    @staticmethod
    def _load(d: str, split: str, ncls: int):
        npy = os.path.join(d, f"{split}_images.npy")
        if os.path.exists(npy):
            x = np.load(npy, allow_pickle=False)
            y = np.load(os.path.join(d, f"{split}_labels.npy"), allow_pickle=False).astype(np.int64)
            if x.ndim == 4 and x.shape[-1] == 3:
                x = x.transpose(0, 3, 1, 2)
            return np.ascontiguousarray(x), y
        if ncls == 100:
            files = [os.path.join(d, "train.bin" if split == "train" else "test.bin")]
            rec, lab_off = 3074, 1           # coarse label, fine label, pixels
        else:
            files = ([os.path.join(d, f"data_batch_{i}.bin") for i in range(1, 6)] if split == "train"
                     else [os.path.join(d, "test_batch.bin")])
            rec, lab_off = 3073, 0
        files = [f for f in files if os.path.exists(f)]
        if not files:
            return None, None
        raw = np.concatenate([np.fromfile(f, dtype=np.uint8) for f in files])
        raw = raw[: len(raw) // rec * rec].reshape(-1, rec)
        y = raw[:, lab_off].astype(np.int64)
        x = raw[:, rec - 3072:].reshape(-1, 3, 32, 32)
        return x, y

    def __len__(self):
        return self.num_batches

    def __iter__(self):
        order = np.random.default_rng(self.seed).permutation(len(self.y))
        mean = self._MEAN[:, None, None]
        std = self._STD[:, None, None]
        for i in range(self.num_batches):
            idx = order[i * self.batch_size:(i + 1) * self.batch_size]
            x = (self.x[idx].astype(np.float32) / 255.0 - mean) / std
            b = {"input": torch.from_numpy(x), "target": torch.from_numpy(self.y[idx])}
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
    if name in ("markov", "markov-lm", "synthetic-markov"):
        return MarkovLanguageModeling(batch_size, seq_len, vocab_size, nb, seed, split, pin_memory=pin_memory)
    if "text" in name or name in ("openwebtext", "wikitext", "tokens", "lm"):
        if native or token_file:
            from ..runtime.native import NativeTokenLoader
            return NativeTokenLoader(batch_size, seq_len, path=token_file, vocab_size=vocab_size,
                                     token_bytes=token_bytes, seed=seed + (0 if split == "train" else 10_000),
                                     num_batches=nb, rank=rank, world=world, pin_memory=pin_memory or None)
        return SyntheticLanguageModeling(batch_size, seq_len, vocab_size, nb, seed, split, data_dir, pin_memory)
    if name in ("cifar10", "cifar-10", "cifar", "cifar100", "cifar-100"):
        ncls = 100 if "100" in name else 10
        if data_dir:
            return ImageArrays(data_dir, batch_size, split, num_batches, seed, ncls, pin_memory)
        return SyntheticImages(batch_size, 32, ncls, nb, seed, split, pin_memory)
    if name in ("imagenet", "imagenet1k", "imagenet-1k"):
        if data_dir:
            return ImageArrays(data_dir, batch_size, split, num_batches, seed, 1000, pin_memory)
        return SyntheticImages(batch_size, 224, 1000, nb, seed, split, pin_memory)
    raise ValueError(f"unknown dataset {dataset_name!r}")
