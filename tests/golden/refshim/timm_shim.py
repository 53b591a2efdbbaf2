"""Restatement of timm's ResNet ``features_only`` trunk (golden generation only).

Follows the structure the reference consumes (transfuser_backbone.py:24-33,50-55,62-65,
175-192,226-239): a ModuleDict-like ``FeatureListNet`` whose ``items()`` yield
conv1, bn1, act1, maxpool, layer1..layer4; ``return_layers`` has 5 entries (stem is a
return layer, so ``start_index = 1``); ``feature_info.info[i]['num_chs'/'reduction']``.
Module / state_dict names follow timm's resnet.py (BasicBlock: conv1, bn1, act1, conv2,
bn2, act2, downsample.{0,1}; Bottleneck adds conv3/bn3/act3, stride on conv2).
``pretrained=True`` is ignored: there is no network here.
"""
from collections import OrderedDict

import torch.nn as nn


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.act1 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.act2 = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        shortcut = x
        x = self.act1(self.bn1(self.conv1(x)))
        x = self.bn2(self.conv2(x))
        if self.downsample is not None:
            shortcut = self.downsample(shortcut)
        return self.act2(x + shortcut)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.act1 = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.act2 = nn.ReLU(inplace=True)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.act3 = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        shortcut = x
        x = self.act1(self.bn1(self.conv1(x)))
        x = self.act2(self.bn2(self.conv2(x)))
        x = self.bn3(self.conv3(x))
        if self.downsample is not None:
            shortcut = self.downsample(shortcut)
        return self.act3(x + shortcut)


_ARCH = {
    "resnet34": (BasicBlock, [3, 4, 6, 3]),
    "resnet50": (Bottleneck, [3, 4, 6, 3]),
}


class _FeatureInfo:
    def __init__(self, info):
        self.info = info

    def channels(self):
        return [i["num_chs"] for i in self.info]


class FeatureListNet(nn.ModuleDict):
    def __init__(self, block, layers, in_chans):
        mods = OrderedDict()
        mods["conv1"] = nn.Conv2d(in_chans, 64, 7, 2, 3, bias=False)
        mods["bn1"] = nn.BatchNorm2d(64)
        mods["act1"] = nn.ReLU(inplace=True)
        mods["maxpool"] = nn.MaxPool2d(3, 2, 1)
        inplanes = 64
        info = [dict(num_chs=64, reduction=2, module="act1")]
        for i, (planes, n) in enumerate(zip([64, 128, 256, 512], layers)):
            stride = 1 if i == 0 else 2
            downsample = None
            if stride != 1 or inplanes != planes * block.expansion:
                downsample = nn.Sequential(
                    nn.Conv2d(inplanes, planes * block.expansion, 1, stride, bias=False),
                    nn.BatchNorm2d(planes * block.expansion))
            blocks = [block(inplanes, planes, stride, downsample)]
            inplanes = planes * block.expansion
            blocks += [block(inplanes, planes) for _ in range(1, n)]
            mods[f"layer{i + 1}"] = nn.Sequential(*blocks)
            info.append(dict(num_chs=inplanes, reduction=4 * 2 ** i, module=f"layer{i + 1}"))
        super().__init__(mods)
        self.return_layers = {m["module"]: m["module"] for m in info}
        self.feature_info = _FeatureInfo(info)


def create_model(name, pretrained=False, features_only=True, in_chans=3, **kwargs):
    assert features_only, "shim only restates features_only trunks"
    block, layers = _ARCH[name]
    return FeatureListNet(block, layers, in_chans)
