"""Compact DARTS search space for FedNAS (reference: `model/cv/darts/*`, 2.5 K LoC).

Mixed operations over a continuous relaxation (softmax over α), normal and
reduction cells, ``arch_parameters()`` / ``new()`` / ``genotype()`` — the
interface FedNAS' trainer/aggregator needs (`mpi_p2p_mp/fednas/FedNASTrainer.py`)."""
from collections import namedtuple

import torch
import torch.nn as nn
import torch.nn.functional as F

Genotype = namedtuple("Genotype", "normal normal_concat reduce reduce_concat")
PRIMITIVES = ["none", "max_pool_3x3", "avg_pool_3x3", "skip_connect", "sep_conv_3x3", "dil_conv_3x3"]


class Zero(nn.Module):
    def __init__(self, stride):
        super().__init__()
        self.stride = stride

    def forward(self, x):
        return x[:, :, :: self.stride, :: self.stride].mul(0.0)


class FactorizedReduce(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.c1 = nn.Conv2d(cin, cout // 2, 1, 2, bias=False)
        self.c2 = nn.Conv2d(cin, cout - cout // 2, 1, 2, bias=False)
        self.bn = nn.BatchNorm2d(cout, affine=False)

    def forward(self, x):
        x = F.relu(x)
        return self.bn(torch.cat([self.c1(x), self.c2(x[:, :, 1:, 1:] if x.shape[-1] > 1 else x)], 1))


def _op(name, c, stride):
    if name == "none":
        return Zero(stride)
    if name == "max_pool_3x3":
        return nn.Sequential(nn.MaxPool2d(3, stride, 1), nn.BatchNorm2d(c, affine=False))
    if name == "avg_pool_3x3":
        return nn.Sequential(nn.AvgPool2d(3, stride, 1, count_include_pad=False), nn.BatchNorm2d(c, affine=False))
    if name == "skip_connect":
        return nn.Identity() if stride == 1 else FactorizedReduce(c, c)
    if name == "sep_conv_3x3":
        return nn.Sequential(nn.ReLU(), nn.Conv2d(c, c, 3, stride, 1, groups=c, bias=False), nn.Conv2d(c, c, 1, bias=False),
                             nn.BatchNorm2d(c, affine=False))
    if name == "dil_conv_3x3":
        return nn.Sequential(nn.ReLU(), nn.Conv2d(c, c, 3, stride, 2, dilation=2, groups=c, bias=False),
                             nn.Conv2d(c, c, 1, bias=False), nn.BatchNorm2d(c, affine=False))
    raise KeyError(name)


class MixedOp(nn.Module):
    def __init__(self, c, stride):
        super().__init__()
        self.ops = nn.ModuleList([_op(p, c, stride) for p in PRIMITIVES])

    def forward(self, x, w):
        return sum(wi * op(x) for wi, op in zip(w, self.ops))


class Cell(nn.Module):
    def __init__(self, steps, multiplier, c_pp, c_p, c, reduction, reduction_prev):
        super().__init__()
        self.reduction = reduction
        self.pre0 = FactorizedReduce(c_pp, c) if reduction_prev else nn.Sequential(nn.ReLU(), nn.Conv2d(c_pp, c, 1, bias=False), nn.BatchNorm2d(c, affine=False))
        self.pre1 = nn.Sequential(nn.ReLU(), nn.Conv2d(c_p, c, 1, bias=False), nn.BatchNorm2d(c, affine=False))
        self.steps = steps
        self.multiplier = multiplier
        self.ops = nn.ModuleList()
        for i in range(steps):
            for j in range(2 + i):
                self.ops.append(MixedOp(c, 2 if reduction and j < 2 else 1))

    def forward(self, s0, s1, weights):
        states = [self.pre0(s0), self.pre1(s1)]
        off = 0
        for i in range(self.steps):
            s = sum(self.ops[off + j](h, weights[off + j]) for j, h in enumerate(states))
            off += len(states)
            states.append(s)
        return torch.cat(states[-self.multiplier:], 1)


class Network(nn.Module):
    def __init__(self, C=8, num_classes=10, layers=3, steps=2, multiplier=2, stem_multiplier=3, criterion=None):
        super().__init__()
        self._C, self._num_classes, self._layers, self._steps, self._multiplier = C, num_classes, layers, steps, multiplier
        self._criterion = criterion or nn.CrossEntropyLoss()
        cc = stem_multiplier * C
        self.stem = nn.Sequential(nn.Conv2d(3, cc, 3, padding=1, bias=False), nn.BatchNorm2d(cc))
        c_pp, c_p, c = cc, cc, C
        self.cells = nn.ModuleList()
        red_prev = False
        for i in range(layers):
            red = i in (layers // 3, 2 * layers // 3)
            if red:
                c *= 2
            cell = Cell(steps, multiplier, c_pp, c_p, c, red, red_prev)
            red_prev = red
            self.cells.append(cell)
            c_pp, c_p = c_p, multiplier * c
        self.pool = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Linear(c_p, num_classes)
        k = sum(2 + i for i in range(steps))
        self.alphas_normal = nn.Parameter(1e-3 * torch.randn(k, len(PRIMITIVES)))
        self.alphas_reduce = nn.Parameter(1e-3 * torch.randn(k, len(PRIMITIVES)))

    def arch_parameters(self):
        return [self.alphas_normal, self.alphas_reduce]

    def weight_parameters(self):
        ids = {id(p) for p in self.arch_parameters()}
        return [p for p in self.parameters() if id(p) not in ids]

    def new(self):
        m = Network(self._C, self._num_classes, self._layers, self._steps, self._multiplier, criterion=self._criterion)
        for a, b in zip(m.arch_parameters(), self.arch_parameters()):
            a.data.copy_(b.data)
        return m

    def forward(self, x):
        s0 = s1 = self.stem(x)
        for cell in self.cells:
            w = F.softmax(self.alphas_reduce if cell.reduction else self.alphas_normal, dim=-1)
            s0, s1 = s1, cell(s0, s1, w)
        return self.classifier(self.pool(s1).flatten(1))

    def _loss(self, x, y):
        return self._criterion(self(x), y)

    def genotype(self):
        def parse(w):
            gene, start, n = [], 0, 2
            for i in range(self._steps):
                W = w[start:start + n]
                edges = sorted(range(i + 2), key=lambda x: -max(W[x][k] for k in range(len(W[x])) if PRIMITIVES[k] != "none"))[:2]
                for j in edges:
                    kb = max((k for k in range(len(W[j])) if PRIMITIVES[k] != "none"), key=lambda k: W[j][k])
                    gene.append((PRIMITIVES[kb], j))
                start += n
                n += 1
            return gene
        concat = list(range(2 + self._steps - self._multiplier, self._steps + 2))
        return Genotype(parse(F.softmax(self.alphas_normal, -1).tolist()), concat,
                        parse(F.softmax(self.alphas_reduce, -1).tolist()), concat)
