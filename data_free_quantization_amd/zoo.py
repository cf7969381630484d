"""Synthetic shape sources for the DFQ weight path: MobileNetV2, ResNet-50 and
DeepLabv3+/MobileNetV2 with the reference's layer shapes and graph structure.

These are NOT the product (the product is the weight-transform path); they exist
so the sweep, the parity tests and the benchmark run on the shapes the reference
quotes (MobileNetV2 53 target layers / 3,469,760 weights,
ResNet-50 54 / 25,502,912, DeepLab 61 / 5,780,288).  Architectures follow
  modeling/classification/MobileNetV2.py:27-129
  modeling/segmentation/backbone/resnet.py:6-124  (+ a torch.mean + Linear head)
  modeling/segmentation/{deeplab,aspp,decoder}.py, backbone/mobilenet.py
Weights are drawn from a numpy PCG64 stream (``init_synthetic``) so the same
tensors can be rebuilt on any machine without the reference or torch's RNG.
"""
from __future__ import annotations

import math
from typing import Iterable

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


# --------------------------------------------------------------------------
# MobileNetV2 (classification)
# --------------------------------------------------------------------------
def _cbr(cin, cout, k, stride, groups=1, act=True, dilation=1, padding=None):
    layers = [
        nn.Conv2d(cin, cout, k, stride, (k // 2) if padding is None else padding, dilation=dilation,
                  groups=groups, bias=False),
        nn.BatchNorm2d(cout),
    ]
    if act:
        layers.append(nn.ReLU6(inplace=True))
    return layers


class _MBBlock(nn.Module):
    """Inverted residual: [pw expand] -> dw 3x3 -> pw linear, residual when shapes allow."""

    def __init__(self, cin, cout, stride, expand):
        super().__init__()
        hidden = int(cin * expand)
        self.residual = stride == 1 and cin == cout
        layers = []
        if expand != 1:
            layers += _cbr(cin, hidden, 1, 1)
        layers += _cbr(hidden, hidden, 3, stride, groups=hidden)
        layers += _cbr(hidden, cout, 1, 1, act=False)
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        if self.residual:
            return x + self.conv(x)
        return self.conv(x)


_MB_SETTING = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2),
               (6, 320, 1, 1)]


class MobileNetV2(nn.Module):
    def __init__(self, n_class=1000):
        super().__init__()
        feats = [nn.Sequential(*_cbr(3, 32, 3, 2))]
        cin = 32
        for t, c, n, s in _MB_SETTING:
            for i in range(n):
                feats.append(_MBBlock(cin, c, s if i == 0 else 1, t))
                cin = c
        feats.append(nn.Sequential(*_cbr(cin, 1280, 1, 1)))
        self.features = nn.Sequential(*feats)
        self.classifier = nn.Linear(1280, n_class)

    def forward(self, x):
        x = self.features(x)
        x = torch.mean(x.view(x.size(0), x.size(1), -1), -1)
        return self.classifier(x)


# --------------------------------------------------------------------------
# ResNet-50 (Bottleneck [3,4,6,3], output stride 16, multi-grid layer4) + head
# --------------------------------------------------------------------------
class _Bottleneck(nn.Module):
    def __init__(self, cin, planes, stride=1, dilation=1, down=None):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, padding=dilation, dilation=dilation, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = down

    def forward(self, x):
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        res = self.downsample(x) if self.downsample is not None else x
        out = out + res
        return self.relu(out)


class ResNet50(nn.Module):
    def __init__(self, n_class=1000):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self._cin = 64
        self.layer1 = self._stage(64, [1, 1, 1], 1)
        self.layer2 = self._stage(128, [1] * 4, 2)
        self.layer3 = self._stage(256, [1] * 6, 2)
        self.layer4 = self._stage(512, [2, 4, 8], 1)   # multi-grid units, dilation 2 * (1, 2, 4)
        self.fc = nn.Linear(2048, n_class)

    def _stage(self, planes, dilations, stride):
        down = None
        if stride != 1 or self._cin != planes * 4:
            down = nn.Sequential(nn.Conv2d(self._cin, planes * 4, 1, stride, bias=False), nn.BatchNorm2d(planes * 4))
        blocks = [_Bottleneck(self._cin, planes, stride, dilations[0], down)]
        self._cin = planes * 4
        blocks += [_Bottleneck(self._cin, planes, 1, d) for d in dilations[1:]]
        return nn.Sequential(*blocks)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.mean(x.view(x.size(0), x.size(1), -1), -1)
        return self.fc(x)


# --------------------------------------------------------------------------
# DeepLabv3+ with a MobileNetV2 backbone (output stride 16)
# --------------------------------------------------------------------------
def _fixed_pad(x, dilation):
    k = 3 + 2 * (dilation - 1)
    lo = (k - 1) // 2
    return F.pad(x, (lo, k - 1 - lo, lo, k - 1 - lo))


class _DLBlock(nn.Module):
    def __init__(self, cin, cout, stride, dilation, expand):
        super().__init__()
        hidden = round(cin * expand)
        self.residual = stride == 1 and cin == cout
        self.dilation = dilation
        layers = []
        if expand != 1:
            layers += _cbr(cin, hidden, 1, 1)
        layers += _cbr(hidden, hidden, 3, stride, groups=hidden, dilation=dilation, padding=0)
        layers += _cbr(hidden, cout, 1, 1, act=False)
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        xp = _fixed_pad(x, self.dilation)
        if self.residual:
            return x + self.conv(xp)
        return self.conv(xp)


class _DLBackbone(nn.Module):
    def __init__(self, output_stride=16):
        super().__init__()
        feats = [nn.Sequential(*_cbr(3, 32, 3, 2, padding=1))]
        cur, rate, cin = 2, 1, 32
        for t, c, n, s in _MB_SETTING:
            if cur == output_stride:
                stride, dil, rate = 1, rate, rate * s
            else:
                stride, dil, cur = s, 1, cur * s
            for i in range(n):
                feats.append(_DLBlock(cin, c, stride if i == 0 else 1, dil, t))
                cin = c
        self.features = nn.Sequential(*feats)

    def forward(self, x):
        low = x
        for i, f in enumerate(self.features):
            x = f(x)
            if i == 3:       # features[0:4] is the low-level branch (backbone/mobilenet.py:115)
                low = x
        return x, low


class _ASPPBranch(nn.Module):
    def __init__(self, cin, k, dilation):
        super().__init__()
        self.atrous_conv = nn.Conv2d(cin, 256, k, 1, 0 if k == 1 else dilation, dilation=dilation, bias=False)
        self.bn = nn.BatchNorm2d(256)
        self.relu = nn.ReLU()

    def forward(self, x):
        return self.relu(self.bn(self.atrous_conv(x)))


class _ASPP(nn.Module):
    def __init__(self, cin=320):
        super().__init__()
        self.aspp1 = _ASPPBranch(cin, 1, 1)
        self.aspp2 = _ASPPBranch(cin, 3, 6)
        self.aspp3 = _ASPPBranch(cin, 3, 12)
        self.aspp4 = _ASPPBranch(cin, 3, 18)
        self.global_avg_pool = nn.Sequential(nn.AdaptiveAvgPool2d((1, 1)), nn.Conv2d(cin, 256, 1, bias=False),
                                             nn.BatchNorm2d(256), nn.ReLU())
        self.conv1 = nn.Conv2d(1280, 256, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(256)
        self.relu = nn.ReLU()
        self.dropout = nn.Dropout(0.5)

    def forward(self, x):
        x1, x2, x3, x4 = self.aspp1(x), self.aspp2(x), self.aspp3(x), self.aspp4(x)
        x5 = F.interpolate(self.global_avg_pool(x), size=x4.size()[2:], mode="bilinear", align_corners=True)
        x = torch.cat((x1, x2, x3, x4, x5), dim=1)
        return self.dropout(self.relu(self.bn1(self.conv1(x))))


class _Decoder(nn.Module):
    def __init__(self, n_class=21, low_in=24):
        super().__init__()
        self.conv1 = nn.Conv2d(low_in, 48, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(48)
        self.relu = nn.ReLU()
        self.last_conv = nn.Sequential(
            nn.Conv2d(304, 256, 3, 1, 1, bias=False), nn.BatchNorm2d(256), nn.ReLU(), nn.Dropout(0.5),
            nn.Conv2d(256, 256, 3, 1, 1, bias=False), nn.BatchNorm2d(256), nn.ReLU(), nn.Dropout(0.1),
            nn.Conv2d(256, n_class, 1, 1))

    def forward(self, x, low):
        low = self.relu(self.bn1(self.conv1(low)))
        x = F.interpolate(x, size=low.size()[2:], mode="bilinear", align_corners=True)
        return self.last_conv(torch.cat((x, low), dim=1))


class DeepLab(nn.Module):
    def __init__(self, n_class=21):
        super().__init__()
        self.backbone = _DLBackbone(16)
        self.aspp = _ASPP(320)
        self.decoder = _Decoder(n_class, 24)

    def forward(self, inp):
        x, low = self.backbone(inp)
        x = self.decoder(self.aspp(x), low)
        return F.interpolate(x, size=inp.size()[2:], mode="bilinear", align_corners=True)


# --------------------------------------------------------------------------
# deterministic synthetic initialisation (SURVEY.md 8d distributions)
# --------------------------------------------------------------------------
def init_synthetic(model: nn.Module, seed: int = 0, kind: str = "mobilenetv2") -> nn.Module:
    """Fill every Conv/Linear/BN tensor from one PCG64 stream, in module order.

    Conv: N(0, sqrt(2/(kh*kw*out))) (MobileNetV2.py:118-120, resnet.py:128-130);
    DeepLab convs: kaiming-normal N(0, sqrt(2/fan_in)); Linear: N(0, 0.01) for
    MobileNetV2 (MobileNetV2.py:126-128), U(+-1/sqrt(fan_in)) otherwise; biases of
    convs that have one: U(+-1/sqrt(fan_in)).  BN stats are randomised so CLE and
    absorption are not degenerate: gamma~U(0.5,1.5), beta~N(0,0.5^2),
    mean~N(0,0.1^2), var~U(0.5,2.0).
    """
    rng = np.random.Generator(np.random.PCG64(seed))

    def put(t: torch.Tensor, a: np.ndarray):
        with torch.no_grad():
            t.copy_(torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).view_as(t))

    for m in model.modules():
        if isinstance(m, nn.Conv2d):
            o, i, kh, kw = m.weight.shape
            if kind == "deeplab":
                std = math.sqrt(2.0 / (i * kh * kw))
            else:
                std = math.sqrt(2.0 / (kh * kw * o))
            put(m.weight, rng.normal(0.0, std, m.weight.shape))
            if m.bias is not None:
                b = 1.0 / math.sqrt(i * kh * kw)
                put(m.bias, rng.uniform(-b, b, m.bias.shape))
        elif isinstance(m, nn.Linear):
            if kind == "mobilenetv2":
                put(m.weight, rng.normal(0.0, 0.01, m.weight.shape))
                put(m.bias, np.zeros(m.bias.shape))
            else:
                b = 1.0 / math.sqrt(m.weight.shape[1])
                put(m.weight, rng.uniform(-b, b, m.weight.shape))
                put(m.bias, rng.uniform(-b, b, m.bias.shape))
        elif isinstance(m, nn.BatchNorm2d):
            c = m.num_features
            put(m.weight, rng.uniform(0.5, 1.5, c))
            put(m.bias, rng.normal(0.0, 0.5, c))
            put(m.running_mean, rng.normal(0.0, 0.1, c))
            put(m.running_var, rng.uniform(0.5, 2.0, c))
    return model


def relu6_to_relu(model: nn.Module) -> nn.Module:
    """The --relu switch (main_dfq.py:156-158): every ReLU6 becomes a ReLU."""
    for name, child in list(model.named_children()):
        if type(child) is nn.ReLU6:
            setattr(model, name, nn.ReLU(inplace=child.inplace))
        else:
            relu6_to_relu(child)
    return model


# --------------------------------------------------------------------------
# ResNet-18: the reference's --resnet model (main_dfq.py:126-128 loads
# torchvision.models.resnet18, absent here).  Module names, shapes and forward
# follow torchvision's ResNet(BasicBlock, [2, 2, 2, 2]) so its checkpoints load
# into it: conv1/bn1/relu/maxpool, layer1..4 of BasicBlocks (downsample.0/.1),
# avgpool, flatten, fc.
# --------------------------------------------------------------------------
class _BasicBlock(nn.Module):
    def __init__(self, cin, planes, stride=1, down=None):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = down

    def forward(self, x):
        identity = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        if self.downsample is not None:
            identity = self.downsample(x)
        out += identity
        return self.relu(out)


class ResNet18(nn.Module):
    def __init__(self, n_class=1000):
        super().__init__()
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self._cin = 64
        self.layer1 = self._stage(64, 1)
        self.layer2 = self._stage(128, 2)
        self.layer3 = self._stage(256, 2)
        self.layer4 = self._stage(512, 2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(512, n_class)

    def _stage(self, planes, stride):
        down = None
        if stride != 1 or self._cin != planes:
            down = nn.Sequential(nn.Conv2d(self._cin, planes, 1, stride, bias=False), nn.BatchNorm2d(planes))
        blocks = [_BasicBlock(self._cin, planes, stride, down), _BasicBlock(planes, planes)]
        self._cin = planes
        return nn.Sequential(*blocks)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        x = torch.flatten(self.avgpool(x), 1)
        return self.fc(x)


MODELS = {"mobilenetv2": MobileNetV2, "resnet50": ResNet50, "deeplab": DeepLab, "resnet18": ResNet18}
INPUT_SHAPES = {"mobilenetv2": (4, 3, 224, 224), "resnet50": (4, 3, 224, 224), "deeplab": (4, 3, 513, 513),
                "resnet18": (4, 3, 224, 224)}


def build(name: str, seed: int = 0, relu: bool = False) -> nn.Module:
    model = MODELS[name]()
    init_synthetic(model, seed, name)
    if relu:
        relu6_to_relu(model)
    return model.eval()


def target_layers(model: nn.Module) -> Iterable[nn.Module]:
    return [m for m in model.modules() if type(m) in (nn.Conv2d, nn.Linear)]
