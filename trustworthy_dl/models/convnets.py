"""VGG-11/13/16 and ResNet-32 (CIFAR) / ResNet-50/101 (ImageNet) as pipeline-layer lists.

README.md:89-92 lists these model families; the reference's ``create_model_partitions`` returns
``{}`` for them (distributed_trainer.py:137-145).  Here every network is expressed as
``pipeline_layers()`` — a flat list of residual blocks / conv units with the classifier (+ loss)
as the last layer — so the same partitioner and pipeline engine run them.  ResNet-32 is the CIFAR
variant (6n+2, n=5; BasicBlocks of 16/32/64 channels), not in torchvision, built here.
On GPU (bf16) every conv+BN(+residual)+ReLU unit runs the native NHWC implicit-GEMM MFMA conv
kernels with fused batch statistics and the one-pass BN/act kernel (ops/conv.py, csrc/conv.hip,
csrc/bn.hip); on CPU the same modules run through torch.  Parameter names are the torchvision ones
(conv1/bn1/..., shortcut.0/shortcut.1), so state dicts are unchanged.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


class ClassifierHead(nn.Module):
    """Global average pool (+ flatten) + FC (+ CE loss when labels are given); last pipeline layer."""
    computes_loss = True

    def __init__(self, in_features: int, num_classes: int, pool: bool = True, hidden: Sequence[int] = ()):
        super().__init__()
        self.pool = pool
        layers: List[nn.Module] = []
        d = in_features
        for hdim in hidden:
            layers += [nn.Linear(d, hdim), nn.ReLU(inplace=True), nn.Dropout(0.0)]
            d = hdim
        layers.append(nn.Linear(d, num_classes))
        self.fc = nn.Sequential(*layers)
        self.num_classes = num_classes

    def forward(self, x, labels=None):
        x = ops.global_avg_pool(x) if self.pool else torch.flatten(x, 1)
        logits = self.fc(x)
        self._last_logits = logits
        if labels is None:
            return logits
        return ops.cross_entropy(logits, labels.reshape(-1), self.num_classes)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin: int, cout: int, stride: int = 1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(cout)
        self.conv2 = nn.Conv2d(cout, cout, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(cout)
        self.shortcut = None
        if stride != 1 or cin != cout:
            self.shortcut = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        sc = x if self.shortcut is None else ops.conv_bn_act(x, self.shortcut[0], self.shortcut[1], relu=False)
        return ops.conv_bn_chain(x, [(self.conv1, self.bn1), (self.conv2, self.bn2)], relu=True, residual=sc)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin: int, width: int, stride: int = 1):
        super().__init__()
        cout = width * 4
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(cout)
        self.shortcut = None
        if stride != 1 or cin != cout:
            self.shortcut = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        sc = x if self.shortcut is None else ops.conv_bn_act(x, self.shortcut[0], self.shortcut[1], relu=False)
        # BN1 + ReLU and BN2 + ReLU are folded into conv2 / conv3 on the native path (never written)
        return ops.conv_bn_chain(x, [(self.conv1, self.bn1), (self.conv2, self.bn2), (self.conv3, self.bn3)],
                                 relu=True, residual=sc)


class Stem(nn.Module):
    def __init__(self, cout: int, imagenet: bool):
        super().__init__()
        if imagenet:
            self.conv = nn.Conv2d(3, cout, 7, 2, 3, bias=False)
        else:
            self.conv = nn.Conv2d(3, cout, 3, 1, 1, bias=False)
        self.bn = nn.BatchNorm2d(cout)
        self.pool = imagenet

    def forward(self, x):
        x = ops.conv_bn_act(x, self.conv, self.bn, relu=True)
        return ops.max_pool2d(x, 3, 2, 1) if self.pool else x


class _PipelineNet(nn.Module):
    family = "cnn"

    def __init__(self, layers: List[nn.Module], input_shape):
        super().__init__()
        self.layers = nn.ModuleList(layers)
        self.input_shape = tuple(input_shape)

    def pipeline_layers(self) -> List[nn.Module]:
        return list(self.layers)

    def forward(self, x, labels=None):
        for layer in self.layers[:-1]:
            x = layer(x)
        return self.layers[-1](x, labels)

    @torch.no_grad()
    def layer_costs(self, batch: int = 1) -> List[float]:
        """MACs per pipeline layer measured with forward hooks on one sample (CPU, eval mode)."""
        costs = []
        x = torch.zeros(batch, *self.input_shape)
        was_training = self.training
        self.eval()
        for layer in self.layers:
            macs = [0.0]

            def hook(m, inp, out):
                if isinstance(m, nn.Conv2d):
                    macs[0] += out.numel() * m.in_channels // m.groups * m.kernel_size[0] * m.kernel_size[1]
                elif isinstance(m, nn.Linear):
                    macs[0] += out.numel() * m.in_features
                elif isinstance(m, (nn.BatchNorm2d,)):
                    macs[0] += 4 * out.numel()

            hs = [m.register_forward_hook(hook) for m in layer.modules()
                  if isinstance(m, (nn.Conv2d, nn.Linear, nn.BatchNorm2d))]
            x = layer(x) if not getattr(layer, "computes_loss", False) else layer(x)
            for h in hs:
                h.remove()
            costs.append(max(macs[0], 1.0))
        self.train(was_training)
        return costs


def _init(model: nn.Module, seed: Optional[int]):
    g = torch.Generator().manual_seed(seed or 0)
    with torch.no_grad():
        for m in model.modules():
            if isinstance(m, nn.Conv2d):
                fan_out = m.out_channels * m.kernel_size[0] * m.kernel_size[1]
                m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (2.0 / fan_out) ** 0.5)
            elif isinstance(m, nn.BatchNorm2d):
                m.weight.fill_(1.0)
                m.bias.zero_()
            elif isinstance(m, nn.Linear):
                bound = 1.0 / m.in_features ** 0.5
                m.weight.copy_((torch.rand(m.weight.shape, generator=g) * 2 - 1) * bound)
                m.bias.zero_()


def resnet_cifar(depth: int = 32, num_classes: int = 10, seed: Optional[int] = 0) -> _PipelineNet:
    assert (depth - 2) % 6 == 0, "CIFAR ResNet depth must be 6n+2"
    n = (depth - 2) // 6
    layers: List[nn.Module] = [Stem(16, imagenet=False)]
    cin = 16
    for i, c in enumerate((16, 32, 64)):
        for j in range(n):
            stride = 2 if (i > 0 and j == 0) else 1
            layers.append(BasicBlock(cin, c, stride))
            cin = c
    layers.append(ClassifierHead(cin, num_classes))
    net = _PipelineNet(layers, (3, 32, 32))
    net.name = f"resnet{depth}"
    _init(net, seed)
    return net


_IMAGENET_DEPTHS = {18: (BasicBlock, (2, 2, 2, 2)), 34: (BasicBlock, (3, 4, 6, 3)),
                    50: (Bottleneck, (3, 4, 6, 3)), 101: (Bottleneck, (3, 4, 23, 3)),
                    152: (Bottleneck, (3, 8, 36, 3))}


def resnet_imagenet(depth: int = 50, num_classes: int = 1000, seed: Optional[int] = 0,
                    image_size: int = 224) -> _PipelineNet:
    block, counts = _IMAGENET_DEPTHS[depth]
    layers: List[nn.Module] = [Stem(64, imagenet=True)]
    cin = 64
    for i, (w, cnt) in enumerate(zip((64, 128, 256, 512), counts)):
        for j in range(cnt):
            stride = 2 if (i > 0 and j == 0) else 1
            layers.append(block(cin, w, stride))
            cin = w * block.expansion
    layers.append(ClassifierHead(cin, num_classes))
    net = _PipelineNet(layers, (3, image_size, image_size))
    net.name = f"resnet{depth}"
    _init(net, seed)
    return net


_VGG_CFGS = {
    11: [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    13: [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
    16: [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
}


class ConvUnit(nn.Module):
    """conv3x3 + BN + ReLU, optionally followed by 2x2 max-pool (a VGG pipeline layer)."""

    def __init__(self, cin: int, cout: int, pool: bool):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, 3, 1, 1, bias=False)
        self.bn = nn.BatchNorm2d(cout)
        self.pool = pool

    def forward(self, x):
        x = ops.conv_bn_act(x, self.conv, self.bn, relu=True)
        return ops.max_pool2d(x, 2) if self.pool else x


def vgg(depth: int = 16, num_classes: int = 10, seed: Optional[int] = 0, image_size: int = 32) -> _PipelineNet:
    cfg = _VGG_CFGS[depth]
    layers: List[nn.Module] = []
    cin = 3
    for i, v in enumerate(cfg):
        if v == "M":
            continue
        pool = i + 1 < len(cfg) and cfg[i + 1] == "M"
        layers.append(ConvUnit(cin, v, pool))
        cin = v
    spatial = image_size // 32
    if image_size >= 224:
        layers.append(ClassifierHead(cin * spatial * spatial, num_classes, pool=False, hidden=(4096, 4096)))
    else:
        layers.append(ClassifierHead(cin, num_classes, pool=True, hidden=(512,)))
    net = _PipelineNet(layers, (3, image_size, image_size))
    net.name = f"vgg{depth}"
    _init(net, seed)
    return net
