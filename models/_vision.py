"""torchvision-compatible image trunks, used when torchvision is not importable.

The reference builds its encoders from torchvision (`vit_b_16`, models/vit_transformer_model.py
:46-52; `resnet101`, models/grid_transformer_model.py:8,44-51).  torchvision is absent from this
image, so these modules restate the published torchvision architectures with IDENTICAL
state_dict key names, so reference checkpoints load unchanged:

  * VisionTransformer(image 224, patch 16, 12 layers, 12 heads, hidden 768, MLP 3072):
    conv_proj, class_token, encoder.pos_embedding, encoder.layers.encoder_layer_{i}.{ln_1,
    self_attention, ln_2, mlp.0, mlp.3}, encoder.ln; pre-LN blocks, LayerNorm eps 1e-6,
    exact-erf GELU.
  * resnet101: Bottleneck v1.5 (stride on the 3x3), layers (3, 4, 23, 3), BN eps 1e-5.

Pretrained weights need the network (ViT_B_16_Weights.DEFAULT / ResNet101_Weights.DEFAULT), so
asking for them raises; load a checkpoint's state_dict instead.
"""
from __future__ import annotations

from collections import OrderedDict

import torch
import torch.nn as nn


class _NoWeights:
    DEFAULT = "DEFAULT"


ViT_B_16_Weights = _NoWeights
ResNet101_Weights = _NoWeights


def _refuse(weights):
    if weights is not None:
        raise RuntimeError("pretrained torchvision weights are unavailable offline; build with "
                           "pretrained=False and load a checkpoint state_dict")


class MLPBlock(nn.Sequential):
    def __init__(self, dim: int, hidden: int):
        super().__init__(nn.Linear(dim, hidden), nn.GELU(), nn.Dropout(0.0), nn.Linear(hidden, dim), nn.Dropout(0.0))


class EncoderBlock(nn.Module):
    def __init__(self, heads: int, dim: int, mlp_dim: int):
        super().__init__()
        self.ln_1 = nn.LayerNorm(dim, eps=1e-6)
        self.self_attention = nn.MultiheadAttention(dim, heads, dropout=0.0, batch_first=True)
        self.dropout = nn.Dropout(0.0)
        self.ln_2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = MLPBlock(dim, mlp_dim)

    def forward(self, x):
        h = self.ln_1(x)
        h, _ = self.self_attention(h, h, h, need_weights=False)
        x = x + self.dropout(h)
        return x + self.mlp(self.ln_2(x))


class Encoder(nn.Module):
    def __init__(self, seq_len: int, layers: int, heads: int, dim: int, mlp_dim: int):
        super().__init__()
        self.pos_embedding = nn.Parameter(torch.empty(1, seq_len, dim).normal_(std=0.02))
        self.dropout = nn.Dropout(0.0)
        self.layers = nn.Sequential(OrderedDict(
            (f"encoder_layer_{i}", EncoderBlock(heads, dim, mlp_dim)) for i in range(layers)))
        self.ln = nn.LayerNorm(dim, eps=1e-6)

    def forward(self, x):
        return self.ln(self.layers(self.dropout(x + self.pos_embedding)))


class VisionTransformer(nn.Module):
    def __init__(self, image_size=224, patch_size=16, num_layers=12, num_heads=12, hidden_dim=768,
                 mlp_dim=3072, num_classes=1000):
        super().__init__()
        self.image_size, self.patch_size, self.hidden_dim = image_size, patch_size, hidden_dim
        self.conv_proj = nn.Conv2d(3, hidden_dim, kernel_size=patch_size, stride=patch_size)
        self.class_token = nn.Parameter(torch.zeros(1, 1, hidden_dim))
        seq = (image_size // patch_size) ** 2 + 1
        self.encoder = Encoder(seq, num_layers, num_heads, hidden_dim, mlp_dim)
        self.heads = nn.Sequential(OrderedDict(head=nn.Linear(hidden_dim, num_classes)))

    def _process_input(self, x):
        n, c, h, w = x.shape
        torch._assert(h == self.image_size and w == self.image_size, "wrong image size")
        g = h // self.patch_size
        x = self.conv_proj(x).reshape(n, self.hidden_dim, g * g)
        return x.permute(0, 2, 1)

    def forward(self, x):
        x = self._process_input(x)
        x = torch.cat([self.class_token.expand(x.shape[0], -1, -1), x], dim=1)
        return self.heads(self.encoder(x)[:, 0])


def vit_b_16(weights=None, **kw):
    _refuse(weights)
    return VisionTransformer(**kw)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        y = self.relu(self.bn1(self.conv1(x)))
        y = self.relu(self.bn2(self.conv2(y)))
        y = self.bn3(self.conv3(y))
        return self.relu(y + (self.downsample(x) if self.downsample is not None else x))


class ResNet(nn.Module):
    def __init__(self, layers=(3, 4, 23, 3), num_classes=1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make(64, layers[0], 1)
        self.layer2 = self._make(128, layers[1], 2)
        self.layer3 = self._make(256, layers[2], 2)
        self.layer4 = self._make(512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(2048, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def _make(self, planes, blocks, stride):
        down = None
        if stride != 1 or self.inplanes != planes * 4:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride=stride, bias=False),
                                 nn.BatchNorm2d(planes * 4))
        mods = [Bottleneck(self.inplanes, planes, stride, down)]
        self.inplanes = planes * 4
        mods += [Bottleneck(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def resnet101(weights=None, **kw):
    _refuse(weights)
    return ResNet((3, 4, 23, 3), **kw)


def load_trunks():
    """(vit_b_16, ViT_B_16_Weights, resnet101, ResNet101_Weights): torchvision's if importable."""
    try:
        from torchvision.models import ResNet101_Weights as RW, ViT_B_16_Weights as VW, resnet101 as r, vit_b_16 as v
        return v, VW, r, RW
    except Exception:
        return vit_b_16, ViT_B_16_Weights, resnet101, ResNet101_Weights
