"""EfficientNet-B0 (reference: `model/cv/efficientnet.py:41-468`), MBConv + SE + swish."""
import math

import torch.nn as nn
import torch.nn.functional as F


class MBConv(nn.Module):
    def __init__(self, cin, cout, k, stride, expand, se_ratio=0.25, drop=0.0):
        super().__init__()
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
        return x + h if self.use_res else h


class EfficientNet(nn.Module):
    # (expand, channels, repeats, stride, kernel)
    B0 = [(1, 16, 1, 1, 3), (6, 24, 2, 2, 3), (6, 40, 2, 2, 5), (6, 80, 3, 2, 3), (6, 112, 3, 1, 5),
          (6, 192, 4, 2, 5), (6, 320, 1, 1, 3)]

    def __init__(self, num_classes=10, width=1.0, depth=1.0, dropout=0.2):
        super().__init__()
        c = lambda v: int(math.ceil(v * width / 8) * 8)
        self.stem = nn.Sequential(nn.Conv2d(3, c(32), 3, 1, 1, bias=False), nn.BatchNorm2d(c(32)), nn.SiLU())
        blocks, cin = [], c(32)
        for e, ch, r, s, k in self.B0:
            for i in range(int(math.ceil(r * depth))):
                blocks.append(MBConv(cin, c(ch), k, s if i == 0 else 1, e))
                cin = c(ch)
        self.blocks = nn.Sequential(*blocks)
        self.head = nn.Sequential(nn.Conv2d(cin, c(1280), 1, bias=False), nn.BatchNorm2d(c(1280)), nn.SiLU())
        self.drop = nn.Dropout(dropout)
        self.fc = nn.Linear(c(1280), num_classes)

    def forward(self, x):
        x = self.head(self.blocks(self.stem(x)))
        return self.fc(self.drop(F.adaptive_avg_pool2d(x, 1).flatten(1)))
