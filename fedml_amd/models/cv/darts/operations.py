"""DARTS candidate operations (reference ``model/cv/darts/operations.py``).

Every op maps (C, stride, affine) → module with C channels in and out; stride 2 halves the spatial
size (the reduction cells' input edges). Separable convs are two ReLU → depthwise → pointwise → BN
stages, dilated convs one such stage with dilation 2 — the channel mixing is in the 1×1 convs, which
is where the FLOPs are."""
import torch
import torch.nn as nn


class Zero(nn.Module):
    def __init__(self, stride):
        super().__init__()
        self.stride = stride

    def forward(self, x):
        return x.mul(0.0) if self.stride == 1 else x[:, :, ::self.stride, ::self.stride].mul(0.0)


class Identity(nn.Module):
    def forward(self, x):
        return x


class ReLUConvBN(nn.Module):
    def __init__(self, cin, cout, k, stride, pad, affine=True):
        super().__init__()
        self.op = nn.Sequential(nn.ReLU(inplace=False), nn.Conv2d(cin, cout, k, stride, pad, bias=False),
                                nn.BatchNorm2d(cout, affine=affine))

    def forward(self, x):
        return self.op(x)


class DilConv(nn.Module):
    def __init__(self, cin, cout, k, stride, pad, dilation, affine=True):
        super().__init__()
        self.op = nn.Sequential(nn.ReLU(inplace=False),
                                nn.Conv2d(cin, cin, k, stride, pad, dilation=dilation, groups=cin, bias=False),
                                nn.Conv2d(cin, cout, 1, bias=False), nn.BatchNorm2d(cout, affine=affine))

    def forward(self, x):
        return self.op(x)


class SepConv(nn.Module):
    """Two stacked (ReLU, depthwise k×k, pointwise, BN) stages; only the first may stride."""

    def __init__(self, cin, cout, k, stride, pad, affine=True):
        super().__init__()
        # one flat Sequential (state_dict keys op.1 … op.7 as in the reference)
        self.op = nn.Sequential(*DilConv(cin, cin, k, stride, pad, 1, affine).op,
                                *DilConv(cin, cout, k, 1, pad, 1, affine).op)

    def forward(self, x):
        return self.op(x)


class FactorizedReduce(nn.Module):
    """Stride-2 channel-preserving shortcut: two 1×1 stride-2 convs on even / odd pixel grids, concatenated."""

    def __init__(self, cin, cout, affine=True):
        super().__init__()
        assert cout % 2 == 0
        self.relu = nn.ReLU(inplace=False)
        self.conv_1 = nn.Conv2d(cin, cout // 2, 1, stride=2, bias=False)
        self.conv_2 = nn.Conv2d(cin, cout // 2, 1, stride=2, bias=False)
        self.bn = nn.BatchNorm2d(cout, affine=affine)

    def forward(self, x):
        x = self.relu(x)
        return self.bn(torch.cat([self.conv_1(x), self.conv_2(x[:, :, 1:, 1:])], 1))


OPS = {
    "none": lambda C, s, a: Zero(s),
    "avg_pool_3x3": lambda C, s, a: nn.AvgPool2d(3, s, 1, count_include_pad=False),
    "max_pool_3x3": lambda C, s, a: nn.MaxPool2d(3, s, 1),
    "skip_connect": lambda C, s, a: Identity() if s == 1 else FactorizedReduce(C, C, a),
    "sep_conv_3x3": lambda C, s, a: SepConv(C, C, 3, s, 1, a),
    "sep_conv_5x5": lambda C, s, a: SepConv(C, C, 5, s, 2, a),
    "sep_conv_7x7": lambda C, s, a: SepConv(C, C, 7, s, 3, a),
    "dil_conv_3x3": lambda C, s, a: DilConv(C, C, 3, s, 2, 2, a),
    "dil_conv_5x5": lambda C, s, a: DilConv(C, C, 5, s, 4, 2, a),
    "conv_7x1_1x7": lambda C, s, a: nn.Sequential(
        nn.ReLU(inplace=False), nn.Conv2d(C, C, (1, 7), (1, s), (0, 3), bias=False),
        nn.Conv2d(C, C, (7, 1), (s, 1), (3, 0), bias=False), nn.BatchNorm2d(C, affine=a)),
}
