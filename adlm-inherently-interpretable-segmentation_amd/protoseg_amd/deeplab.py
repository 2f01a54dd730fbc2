"""DeepLabV2-ResNet101 backbone + MSC wrapper (stays on PyTorch-ROCm; not on the HIP hot path).

The reference imports ``deeplab_pytorch.libs.models.deeplabv2.DeepLabV2`` from an un-vendored
submodule (reference .gitmodules:1-3; deeplab_features.py:5, 52-60). This is a fresh
implementation of that public architecture with the module names the reference relies on:
  * ``layer{1..5}.block{i}.{reduce,conv3x3,increase,shortcut}.{conv,bn}`` and
    ``layer1.conv1.{conv,bn}`` — the ImageNet key remap of deeplab_features.py:8-49;
  * ``aspp.c0..c3.{weight,bias}`` — optimizer groups of module.py:336-343 and
    train_and_test.py:157-166;
  * ``freeze_bn()`` — module.py:127, 278.
Output stride 8 (layer4/5 dilated 2/4), ceil-mode stem pool: 513x513 -> 65x65 and
1024x2048 -> 129x257 (push.py:275).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F


class ConvBnReLU(nn.Sequential):
    def __init__(self, in_ch: int, out_ch: int, kernel_size: int, stride: int, padding: int, dilation: int,
                 relu: bool = True):
        super().__init__()
        self.add_module("conv", nn.Conv2d(in_ch, out_ch, kernel_size, stride, padding, dilation, bias=False))
        self.add_module("bn", nn.BatchNorm2d(out_ch, eps=1e-5, momentum=0.001))
        if relu:
            self.add_module("relu", nn.ReLU())


class Bottleneck(nn.Module):
    def __init__(self, in_ch: int, out_ch: int, stride: int, dilation: int, downsample: bool):
        super().__init__()
        mid = out_ch // 4
        self.reduce = ConvBnReLU(in_ch, mid, 1, stride, 0, 1, True)
        self.conv3x3 = ConvBnReLU(mid, mid, 3, 1, dilation, dilation, True)
        self.increase = ConvBnReLU(mid, out_ch, 1, 1, 0, 1, False)
        self.shortcut = ConvBnReLU(in_ch, out_ch, 1, stride, 0, 1, False) if downsample else None

    def forward(self, x):
        h = self.increase(self.conv3x3(self.reduce(x)))
        return F.relu(h + (self.shortcut(x) if self.shortcut is not None else x))


class ResLayer(nn.Sequential):
    def __init__(self, n_blocks: int, in_ch: int, out_ch: int, stride: int, dilation: int):
        super().__init__()
        for i in range(n_blocks):
            self.add_module(f"block{i + 1}", Bottleneck(in_ch if i == 0 else out_ch, out_ch,
                                                         stride if i == 0 else 1, dilation, i == 0))


class Stem(nn.Sequential):
    def __init__(self, out_ch: int):
        super().__init__()
        self.add_module("conv1", ConvBnReLU(3, out_ch, 7, 2, 3, 1))
        self.add_module("pool", nn.MaxPool2d(3, 2, 1, ceil_mode=True))


class ASPP(nn.Module):
    """Atrous spatial pyramid pooling: the sum of dilated 3x3 branches."""

    def __init__(self, in_ch: int, out_ch: int, rates: Sequence[int]):
        super().__init__()
        for i, rate in enumerate(rates):
            self.add_module(f"c{i}", nn.Conv2d(in_ch, out_ch, 3, 1, padding=rate, dilation=rate, bias=True))
        for m in self.children():
            nn.init.normal_(m.weight, mean=0, std=0.01)
            nn.init.constant_(m.bias, 0)

    def forward(self, x):
        out = None
        for stage in self.children():
            y = stage(x)
            out = y if out is None else out + y
        return out


class DeepLabV2(nn.Sequential):
    """ResNet-101 (n_blocks [3, 4, 23, 3]) with ASPP rates [6, 12, 18, 24] (deeplab_features.py:56-57)."""

    def __init__(self, n_classes: int, n_blocks: Sequence[int], atrous_rates: Sequence[int]):
        super().__init__()
        ch = [64 * 2 ** p for p in range(6)]
        self.add_module("layer1", Stem(ch[0]))
        self.add_module("layer2", ResLayer(n_blocks[0], ch[0], ch[2], 1, 1))
        self.add_module("layer3", ResLayer(n_blocks[1], ch[2], ch[3], 2, 1))
        self.add_module("layer4", ResLayer(n_blocks[2], ch[3], ch[4], 1, 2))
        self.add_module("layer5", ResLayer(n_blocks[3], ch[4], ch[5], 1, 4))
        self.add_module("aspp", ASPP(ch[5], n_classes, atrous_rates))

    def freeze_bn(self):
        for m in self.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.eval()


class MSC(nn.Module):
    """Multi-scale inputs with pixel-wise max (segmentation/utils.py:64-101)."""

    def __init__(self, base: nn.Module, scales: Optional[List[float]] = None):
        super().__init__()
        self.base = base
        self.scales = scales if scales is not None else [0.5, 0.75]

    def forward(self, x):
        logits = self.base(x)
        if len(self.scales) == 0:
            return logits
        _, _, H, W = logits.shape
        pyramid = [self.base(F.interpolate(x, scale_factor=p, mode="bilinear", align_corners=False))
                   for p in self.scales]
        interp = [F.interpolate(l, size=(H, W), mode="bilinear", align_corners=False) for l in pyramid]
        logits_max = torch.max(torch.stack([logits] + interp), dim=0)[0]
        if self.training:
            return [logits] + pyramid + [logits_max]
        return logits_max


def deeplabv2_resnet101_features(pretrained: bool = False, deeplab_n_features: int = 64,
                                 scales: Optional[List[float]] = None, n_blocks: Sequence[int] = (3, 4, 23, 3),
                                 **kwargs) -> MSC:
    """deeplab_features.py:52-60. ``pretrained`` weights need the network (train.py:82) and are
    loaded by the caller; ``n_blocks`` is exposed only so tests can build a shallow variant."""
    return MSC(base=DeepLabV2(n_classes=deeplab_n_features, n_blocks=list(n_blocks), atrous_rates=[6, 12, 18, 24]),
               scales=[1.0] if scales is None else scales)
