"""Stand-in ``torchvision`` modules used ONLY by make_golden.py to let the reference module
``misinfo_forensics.py`` import in the build container (torchvision is not installed;
SURVEY.md §8c).  ``efficientnet_b0`` is an independent nn.Module restatement of torchvision's
EfficientNet-B0 (same module tree / state-dict names), so the reference's own
``forward_image`` / ``analyze_image`` code runs; EfficientNet numbers in the fixtures are
therefore "parity vs torchvision unpinned" (structure pinned: 5,288,548 params at 1000
classes, 360 state-dict keys).  ``transforms`` restates Resize/ToTensor/Normalize/Compose.
"""
from __future__ import annotations

import sys
import types

import numpy as np
import torch
import torch.nn as nn

_SETTING = [(1, 3, 1, 32, 16, 1), (6, 3, 2, 16, 24, 2), (6, 5, 2, 24, 40, 2), (6, 3, 2, 40, 80, 3),
            (6, 5, 1, 80, 112, 3), (6, 5, 2, 112, 192, 4), (6, 3, 1, 192, 320, 1)]


def _cna(cin, cout, k, s=1, groups=1, act=True):
    layers = [nn.Conv2d(cin, cout, k, s, (k - 1) // 2, groups=groups, bias=False), nn.BatchNorm2d(cout)]
    if act:
        layers.append(nn.SiLU(inplace=True))
    return nn.Sequential(*layers)


class _SE(nn.Module):
    def __init__(self, c, sq):
        super().__init__()
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc1 = nn.Conv2d(c, sq, 1)
        self.fc2 = nn.Conv2d(sq, c, 1)
        self.activation = nn.SiLU()
        self.scale_activation = nn.Sigmoid()

    def forward(self, x):
        s = self.scale_activation(self.fc2(self.activation(self.fc1(self.avgpool(x)))))
        return s * x


class _MBConv(nn.Module):
    def __init__(self, e, k, s, cin, cout):
        super().__init__()
        self.use_res = s == 1 and cin == cout
        cexp = cin * e
        layers = []
        if cexp != cin:
            layers.append(_cna(cin, cexp, 1))
        layers.append(_cna(cexp, cexp, k, s, groups=cexp))
        layers.append(_SE(cexp, max(1, cin // 4)))
        layers.append(_cna(cexp, cout, 1, act=False))
        self.block = nn.Sequential(*layers)

    def forward(self, x):
        y = self.block(x)
        return y + x if self.use_res else y


class EfficientNetB0(nn.Module):
    def __init__(self, num_classes=1000):
        super().__init__()
        feats = [_cna(3, 32, 3, 2)]
        for e, k, s, cin, cout, n in _SETTING:
            feats.append(nn.Sequential(*[_MBConv(e, k, s if j == 0 else 1, cin if j == 0 else cout, cout)
                                         for j in range(n)]))
        feats.append(_cna(320, 1280, 1))
        self.features = nn.Sequential(*feats)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Sequential(nn.Dropout(0.2, inplace=True), nn.Linear(1280, num_classes))

    def forward(self, x):
        return self.classifier(torch.flatten(self.avgpool(self.features(x)), 1))


def efficientnet_b0(weights=None, **kw):
    assert weights is None
    return EfficientNetB0(**kw)


class Compose:
    def __init__(self, ts):
        self.ts = ts

    def __call__(self, x):
        for t in self.ts:
            x = t(x)
        return x


class Resize:
    def __init__(self, size):
        self.size = size

    def __call__(self, img):
        from PIL import Image
        h, w = self.size
        return img.resize((w, h), Image.BILINEAR)


class ToTensor:
    def __call__(self, img):
        a = torch.from_numpy(np.array(img, dtype=np.uint8, copy=True))
        return a.permute(2, 0, 1).contiguous().to(torch.float32).div(255)


class Normalize:
    def __init__(self, mean, std):
        self.mean, self.std = mean, std

    def __call__(self, t):
        m = torch.as_tensor(self.mean, dtype=t.dtype).view(-1, 1, 1)
        s = torch.as_tensor(self.std, dtype=t.dtype).view(-1, 1, 1)
        return t.sub(m).div(s)


def install():
    """Register stub ``dotenv`` and ``torchvision`` packages in sys.modules."""
    dotenv = types.ModuleType("dotenv")
    dotenv.load_dotenv = lambda *a, **k: False
    tv = types.ModuleType("torchvision")
    models = types.ModuleType("torchvision.models")
    models.efficientnet_b0 = efficientnet_b0
    transforms = types.ModuleType("torchvision.transforms")
    for c in (Compose, Resize, ToTensor, Normalize):
        setattr(transforms, c.__name__, c)
    tv.models, tv.transforms = models, transforms
    sys.modules.update({"dotenv": dotenv, "torchvision": tv, "torchvision.models": models,
                        "torchvision.transforms": transforms})
