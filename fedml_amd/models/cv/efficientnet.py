"""EfficientNet-B0…B7 (reference: `model/cv/efficientnet.py:41-468`, `efficientnet_utils.py`): MBConv + SE +
swish, compound scaling of width / depth / resolution (``EfficientNet.from_name("efficientnet-b3")``),
drop-connect (stochastic depth) growing linearly with block index as in the reference."""
import math

import torch.nn as nn
import torch.nn.functional as F


import torch

# (width, depth, resolution, dropout) per variant (efficientnet_utils.py efficientnet_params)
PARAMS = {"efficientnet-b0": (1.0, 1.0, 224, 0.2), "efficientnet-b1": (1.0, 1.1, 240, 0.2),
          "efficientnet-b2": (1.1, 1.2, 260, 0.3), "efficientnet-b3": (1.2, 1.4, 300, 0.3),
          "efficientnet-b4": (1.4, 1.8, 380, 0.4), "efficientnet-b5": (1.6, 2.2, 456, 0.4),
          "efficientnet-b6": (1.8, 2.6, 528, 0.5), "efficientnet-b7": (2.0, 3.1, 600, 0.5)}


def round_filters(f, width, divisor=8):
    """Channel count scaled by ``width``, rounded to a multiple of 8, never below 90 % of the scaled value."""
    if width == 1.0:
        return f
    f = f * width
    new = max(divisor, int(f + divisor / 2) // divisor * divisor)
    if new < 0.9 * f:
        new += divisor
    return int(new)


def drop_connect(x, p, training):
    if not training or p <= 0.0:
        return x
    keep = 1.0 - p
    mask = torch.floor(keep + torch.rand(x.shape[0], 1, 1, 1, device=x.device, dtype=x.dtype))
    return x / keep * mask


class MBConv(nn.Module):
    def __init__(self, cin, cout, k, stride, expand, se_ratio=0.25, drop=0.0):
        super().__init__()
        self.drop = drop
        mid = cin * expand
        self.use_res = stride == 1 and cin == cout
        self.expand = nn.Sequential(nn.Conv2d(cin, mid, 1, bias=False), nn.BatchNorm2d(mid), nn.SiLU()) if expand != 1 else nn.Identity()
        self.dw = nn.Sequential(nn.Conv2d(mid, mid, k, stride, k // 2, groups=mid, bias=False), nn.BatchNorm2d(mid), nn.SiLU())
        sq = max(1, int(cin * se_ratio))
        self.se1 = nn.Conv2d(mid, sq, 1)
        self.se2 = nn.Conv2d(sq, mid, 1)
        self.project = nn.Sequential(nn.Conv2d(mid, cout, 1, bias=False), nn.BatchNorm2d(cout))

    def forward(self, x):
        h = self.dw(self.expand(x))
        s = F.adaptive_avg_pool2d(h, 1)
        h = h * self.se2(F.silu(self.se1(s))).sigmoid()
        h = self.project(h)
        return x + drop_connect(h, self.drop, self.training) if self.use_res else h


class EfficientNet(nn.Module):
    # (expand, channels, repeats, stride, kernel)
    B0 = [(1, 16, 1, 1, 3), (6, 24, 2, 2, 3), (6, 40, 2, 2, 5), (6, 80, 3, 2, 3), (6, 112, 3, 1, 5),
          (6, 192, 4, 2, 5), (6, 320, 1, 1, 3)]

    def __init__(self, num_classes=10, width=1.0, depth=1.0, dropout=0.2, drop_connect_rate=0.0, stem_stride=1):
        super().__init__()
        c = lambda v: round_filters(v, width)
        self.stem = nn.Sequential(nn.Conv2d(3, c(32), 3, stem_stride, 1, bias=False), nn.BatchNorm2d(c(32)), nn.SiLU())
        reps = [int(math.ceil(r * depth)) for _, _, r, _, _ in self.B0]
        total, idx = sum(reps), 0
        blocks, cin = [], c(32)
        for (e, ch, r, s, k), n in zip(self.B0, reps):
            for i in range(n):
                blocks.append(MBConv(cin, c(ch), k, s if i == 0 else 1, e, drop=drop_connect_rate * idx / total))
                cin = c(ch)
                idx += 1
        self.blocks = nn.Sequential(*blocks)
        self.head = nn.Sequential(nn.Conv2d(cin, c(1280), 1, bias=False), nn.BatchNorm2d(c(1280)), nn.SiLU())
        self.drop = nn.Dropout(dropout)
        self.fc = nn.Linear(c(1280), num_classes)

    @classmethod
    def from_name(cls, name, num_classes=1000, drop_connect_rate=0.2, **kw):
        """``efficientnet-b0`` … ``b7`` (ImageNet stem stride 2); ``image_size`` = PARAMS[name][2]."""
        w, d, _, p = PARAMS[name]
        return cls(num_classes, w, d, p, drop_connect_rate, stem_stride=kw.pop("stem_stride", 2), **kw)

    def forward(self, x):
        x = self.head(self.blocks(self.stem(x)))
        return self.fc(self.drop(F.adaptive_avg_pool2d(x, 1).flatten(1)))
