"""Segmentation networks for FedSeg: a DeepLabV3+-style net (ResNet trunk, ASPP, low-level
decoder) and a small UNet. The reference's FedSeg (`mpi_p2p_mp/fedseg`) takes DeepLabV3+/UNet
from its model zoo; these are compact re-designs with the same input/output contract
(``[B,3,H,W] → [B,n_classes,H,W]`` logits)."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .resnet import BasicBlock


def _cbr(cin, cout, k=3, d=1):
    return nn.Sequential(nn.Conv2d(cin, cout, k, padding=d * (k // 2), dilation=d, bias=False), nn.BatchNorm2d(cout),
                         nn.ReLU(inplace=True))


class ASPP(nn.Module):
    def __init__(self, cin, cout, rates=(1, 6, 12, 18)):
        super().__init__()
        self.branches = nn.ModuleList([_cbr(cin, cout, 1 if r == 1 else 3, r) for r in rates])
        self.pool = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(cin, cout, 1, bias=False), nn.ReLU(inplace=True))
        self.project = _cbr(cout * (len(rates) + 1), cout, 1)

    def forward(self, x):
        feats = [b(x) for b in self.branches]
        feats.append(self.pool(x).expand(-1, -1, x.shape[2], x.shape[3]))
        return self.project(torch.cat(feats, 1))


class DeepLabV3Plus(nn.Module):
    def __init__(self, n_classes=21, width=32, blocks=(2, 2, 2)):
        super().__init__()
        self.n_classes = n_classes
        w = width
        self.stem = _cbr(3, w)
        self.layer1 = nn.Sequential(*[BasicBlock(w, w, 2 if i == 0 else 1,
                                                 nn.Sequential(nn.Conv2d(w, w, 1, 2, bias=False), nn.BatchNorm2d(w))
                                                 if i == 0 else None) for i in range(blocks[0])])
        self.layer2 = nn.Sequential(*[BasicBlock(w if i == 0 else 2 * w, 2 * w, 2 if i == 0 else 1,
                                                 nn.Sequential(nn.Conv2d(w, 2 * w, 1, 2, bias=False),
                                                               nn.BatchNorm2d(2 * w)) if i == 0 else None)
                                      for i in range(blocks[1])])
        self.layer3 = nn.Sequential(*[BasicBlock(2 * w if i == 0 else 4 * w, 4 * w, 1,
                                                 nn.Sequential(nn.Conv2d(2 * w, 4 * w, 1, bias=False),
                                                               nn.BatchNorm2d(4 * w)) if i == 0 else None)
                                      for i in range(blocks[2])])
        self.aspp = ASPP(4 * w, 4 * w, (1, 2, 4, 6))
        self.low = _cbr(w, w // 2, 1)
        self.decoder = nn.Sequential(_cbr(4 * w + w // 2, 2 * w), _cbr(2 * w, 2 * w), nn.Conv2d(2 * w, n_classes, 1))

    def forward(self, x):
        h, w_ = x.shape[2:]
        low = self.layer1(self.stem(x))
        hi = self.aspp(self.layer3(self.layer2(low)))
        hi = F.interpolate(hi, size=low.shape[2:], mode="bilinear", align_corners=False)
        out = self.decoder(torch.cat([hi, self.low(low)], 1))
        return F.interpolate(out, size=(h, w_), mode="bilinear", align_corners=False)


class UNet(nn.Module):
    def __init__(self, n_classes=21, width=16, depth=3):
        super().__init__()
        self.n_classes = n_classes
        self.downs = nn.ModuleList()
        c, chans = 3, []
        for i in range(depth):
            self.downs.append(nn.Sequential(_cbr(c, width << i), _cbr(width << i, width << i)))
            chans.append(width << i)
            c = width << i
        self.mid = nn.Sequential(_cbr(c, c * 2), _cbr(c * 2, c * 2))
        c = c * 2
        self.ups = nn.ModuleList()
        self.up_convs = nn.ModuleList()
        for ch in reversed(chans):
            self.ups.append(nn.ConvTranspose2d(c, ch, 2, 2))
            self.up_convs.append(nn.Sequential(_cbr(2 * ch, ch), _cbr(ch, ch)))
            c = ch
        self.head = nn.Conv2d(c, n_classes, 1)

    def forward(self, x):
        skips = []
        for d in self.downs:
            x = d(x)
            skips.append(x)
            x = F.max_pool2d(x, 2)
        x = self.mid(x)
        for up, conv, s in zip(self.ups, self.up_convs, reversed(skips)):
            x = conv(torch.cat([up(x), s], 1))
        return self.head(x)
