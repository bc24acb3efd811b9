"""Model zoo entry points: ``ModelFactory().create_model(name)`` (distributed_trainer.py:118-119)
and ``get_model(name)`` (README.md:60).  Names: gpt2[-tiny|-mini|-small|-medium|-large|-xl],
resnet32 (CIFAR), resnet18/34/50/101/152 (ImageNet), vgg11/13/16 (CIFAR; ``-imagenet`` suffix
for 224x224 inputs)."""
from __future__ import annotations

import re
from typing import Optional

import torch.nn as nn

from .convnets import resnet_cifar, resnet_imagenet, vgg
from .gpt2 import GPT2Config, GPT2LMHeadModel

SUPPORTED = ["gpt2", "gpt2-tiny", "gpt2-mini", "gpt2-small", "gpt2-medium", "gpt2-large", "gpt2-xl",
             "resnet20", "resnet32", "resnet44", "resnet56", "resnet110", "resnet18", "resnet34", "resnet50",
             "resnet101", "resnet152", "vgg11", "vgg13", "vgg16"]


def get_model(name: str, size: Optional[str] = None, num_classes: Optional[int] = None, seed: int = 0,
              seq_len: Optional[int] = None, image_size: Optional[int] = None, **kw) -> nn.Module:
    n = name.lower().replace("_", "-")
    if n.startswith("gpt2"):
        sz = size or (n.split("-", 1)[1] if "-" in n else "small")
        extra = {}
        if seq_len is not None:
            extra["n_positions"] = max(seq_len, 1)
        extra.update(kw)
        model = GPT2LMHeadModel(GPT2Config.from_size(sz, **extra), seed=seed)
        model.name = f"gpt2-{sz}"
        return model
    m = re.match(r"resnet(\d+)(-imagenet|-cifar)?", n)
    if m:
        depth = int(m.group(1))
        if depth in (18, 34, 50, 101, 152) and m.group(2) != "-cifar":
            return resnet_imagenet(depth, num_classes or 1000, seed, image_size or 224)
        return resnet_cifar(depth, num_classes or 10, seed)
    m = re.match(r"vgg(\d+)(-imagenet)?", n)
    if m:
        imgs = image_size or (224 if m.group(2) else 32)
        return vgg(int(m.group(1)), num_classes or (1000 if imgs >= 224 else 10), seed, imgs)
    raise ValueError(f"unknown model {name!r}; supported: {SUPPORTED}")


class ModelFactory:
    """Reference-compatible factory (phantom models/model_factory.py)."""

    def create_model(self, model_name: str, **kw) -> nn.Module:
        return get_model(model_name, **kw)

    @staticmethod
    def supported_models():
        return list(SUPPORTED)
