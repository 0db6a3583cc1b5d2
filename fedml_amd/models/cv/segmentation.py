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


# ---------------------------------------------------------------------------------------------------
# DeepLabV3+ with the reference FedSeg's backbones (ResNet-50/101 with output stride 16/8 via dilation,
# MobileNetV2) — reference: FedSeg's `model_trainer` contract (`mpi_p2p_mp/fedseg/MyModelTrainer.py`):
# ``encoder_decoder`` (ASPP + decoder) is what travels when ``backbone_freezed``; the backbone trains at
# 1× and the head at 10× the learning rate (``get_1x_lr_params`` / ``get_10x_lr_params``).
# ---------------------------------------------------------------------------------------------------
class _Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, planes, stride=1, dilation=1, down=None):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, dilation, dilation, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.down = down

    def forward(self, x):
        idt = x if self.down is None else self.down(x)
        y = F.relu(self.bn1(self.conv1(x)), inplace=True)
        y = F.relu(self.bn2(self.conv2(y)), inplace=True)
        return F.relu(self.bn3(self.conv3(y)) + idt, inplace=True)


class ResNetBackbone(nn.Module):
    """ResNet-50/101 trunk; output stride 16 (layer4 dilated 2) or 8 (layer3 dilated 2, layer4 4).
    Returns (high-level features [2048 ch], low-level features from layer1 [256 ch])."""

    def __init__(self, layers=(3, 4, 23, 3), output_stride=16):
        super().__init__()
        strides, dil = ((1, 2, 2, 1), (1, 1, 1, 2)) if output_stride == 16 else ((1, 2, 1, 1), (1, 1, 2, 4))
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.inplanes = 64
        self.layer1 = self._make(64, layers[0], strides[0], dil[0])
        self.layer2 = self._make(128, layers[1], strides[1], dil[1])
        self.layer3 = self._make(256, layers[2], strides[2], dil[2])
        self.layer4 = self._make(512, layers[3], strides[3], dil[3], multi_grid=(1, 2, 4))
        self.out_channels, self.low_channels = 2048, 256

    def _make(self, planes, n, stride, dilation, multi_grid=None):
        down = None
        if stride != 1 or self.inplanes != planes * 4:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride, bias=False), nn.BatchNorm2d(planes * 4))
        blocks = []
        for i in range(n):
            d = dilation * (multi_grid[i % len(multi_grid)] if multi_grid else 1)
            blocks.append(_Bottleneck(self.inplanes, planes, stride if i == 0 else 1, d, down if i == 0 else None))
            self.inplanes = planes * 4
        return nn.Sequential(*blocks)

    def forward(self, x):
        x = F.max_pool2d(F.relu(self.bn1(self.conv1(x)), inplace=True), 3, 2, 1)
        low = self.layer1(x)
        return self.layer4(self.layer3(self.layer2(low))), low


class _InvRes(nn.Module):
    def __init__(self, cin, cout, stride, expand, dilation=1):
        super().__init__()
        hid = cin * expand
        self.use_res = stride == 1 and cin == cout
        layers = [] if expand == 1 else [nn.Conv2d(cin, hid, 1, bias=False), nn.BatchNorm2d(hid), nn.ReLU6(True)]
        layers += [nn.Conv2d(hid, hid, 3, stride, dilation, dilation, groups=hid, bias=False), nn.BatchNorm2d(hid),
                   nn.ReLU6(True), nn.Conv2d(hid, cout, 1, bias=False), nn.BatchNorm2d(cout)]
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        return x + self.conv(x) if self.use_res else self.conv(x)


class MobileNetV2Backbone(nn.Module):
    """MobileNetV2 trunk at output stride 16 (the last stride-2 stage dilated); low-level features after
    the stride-4 stage (24 ch), high-level 320 ch."""

    def __init__(self, output_stride=16):
        super().__init__()
        cfg = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2), (6, 320, 1, 1)]
        self.stem = nn.Sequential(nn.Conv2d(3, 32, 3, 2, 1, bias=False), nn.BatchNorm2d(32), nn.ReLU6(True))
        feats, cin, cur_stride, dil = [], 32, 2, 1
        self.low_idx = None
        for t, c, n, s in cfg:
            if cur_stride >= output_stride and s == 2:
                dil *= s
                s = 1
            else:
                cur_stride *= s
            for i in range(n):
                feats.append(_InvRes(cin, c, s if i == 0 else 1, t, dil))
                cin = c
            if c == 24:
                self.low_idx = len(feats)
        self.features = nn.Sequential(*feats)
        self.out_channels, self.low_channels = 320, 24

    def forward(self, x):
        x = self.stem(x)
        low = self.features[:self.low_idx](x)
        return self.features[self.low_idx:](low), low


class _EncoderDecoder(nn.Module):
    """ASPP (rates by output stride) + the DeepLabV3+ decoder (48-ch low-level projection)."""

    def __init__(self, cin, clow, n_classes, output_stride=16):
        super().__init__()
        rates = (1, 6, 12, 18) if output_stride == 16 else (1, 12, 24, 36)
        self.aspp = ASPP(cin, 256, rates)
        self.low = _cbr(clow, 48, 1)
        self.decoder = nn.Sequential(_cbr(256 + 48, 256), _cbr(256, 256), nn.Conv2d(256, n_classes, 1))

    def forward(self, high, low):
        hi = F.interpolate(self.aspp(high), size=low.shape[2:], mode="bilinear", align_corners=False)
        return self.decoder(torch.cat([hi, self.low(low)], 1))


class DeepLabV3PlusNet(nn.Module):
    def __init__(self, n_classes=21, backbone="resnet101", output_stride=16, backbone_freezed=False):
        super().__init__()
        self.n_classes = n_classes
        if backbone in ("resnet101", "resnet"):
            self.backbone = ResNetBackbone((3, 4, 23, 3), output_stride)
        elif backbone == "resnet50":
            self.backbone = ResNetBackbone((3, 4, 6, 3), output_stride)
        elif backbone == "mobilenet":
            self.backbone = MobileNetV2Backbone(output_stride)
        else:
            raise ValueError(f"backbone {backbone!r}: resnet101 | resnet50 | mobilenet")
        self.encoder_decoder = _EncoderDecoder(self.backbone.out_channels, self.backbone.low_channels, n_classes,
                                               output_stride)
        if backbone_freezed:
            for p in self.backbone.parameters():
                p.requires_grad_(False)

    def forward(self, x):
        high, low = self.backbone(x)
        return F.interpolate(self.encoder_decoder(high, low), size=x.shape[2:], mode="bilinear", align_corners=False)

    def get_1x_lr_params(self):
        return [p for p in self.backbone.parameters() if p.requires_grad]

    def get_10x_lr_params(self):
        return [p for p in self.encoder_decoder.parameters() if p.requires_grad]
