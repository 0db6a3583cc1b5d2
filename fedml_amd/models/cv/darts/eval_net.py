"""Genotype-built evaluation network for FedNAS ``stage: train`` (reference ``model/cv/darts/model.py``):
each cell has exactly the two chosen operations per node, drop-path regularisation on non-identity
edges, and an auxiliary classifier after the second reduction cell. ``forward`` returns
(logits, auxiliary logits | None)."""
import torch
import torch.nn as nn

from . import genotypes
from .operations import OPS, FactorizedReduce, Identity, ReLUConvBN


def drop_path(x, drop_prob: float):
    """Drop whole samples of an edge's output with probability p, scaling the kept ones by 1/(1 − p)."""
    if drop_prob <= 0.0:
        return x
    keep = 1.0 - drop_prob
    mask = torch.empty(x.shape[0], 1, 1, 1, device=x.device, dtype=x.dtype).bernoulli_(keep)
    return x / keep * mask


class EvalCell(nn.Module):
    def __init__(self, genotype, c_pp, c_p, c, reduction, reduction_prev):
        super().__init__()
        self.preprocess0 = FactorizedReduce(c_pp, c) if reduction_prev else ReLUConvBN(c_pp, c, 1, 1, 0)
        self.preprocess1 = ReLUConvBN(c_p, c, 1, 1, 0)
        names, idx = zip(*(genotype.reduce if reduction else genotype.normal))
        self._concat = list(genotype.reduce_concat if reduction else genotype.normal_concat)
        self.multiplier = len(self._concat)
        self._steps = len(names) // 2
        self._indices = idx
        self._ops = nn.ModuleList(OPS[n](c, 2 if reduction and i < 2 else 1, True) for n, i in zip(names, idx))

    def forward(self, s0, s1, drop_prob):
        states = [self.preprocess0(s0), self.preprocess1(s1)]
        for i in range(self._steps):
            hs = []
            for e in (2 * i, 2 * i + 1):
                h = self._ops[e](states[self._indices[e]])
                if self.training and drop_prob > 0.0 and not isinstance(self._ops[e], Identity):
                    h = drop_path(h, drop_prob)
                hs.append(h)
            states.append(hs[0] + hs[1])
        return torch.cat([states[i] for i in self._concat], 1)


class AuxiliaryHeadCIFAR(nn.Module):
    """Auxiliary classifier on the 8×8 feature map after the second reduction (→ 2×2 → 768 features)."""

    def __init__(self, c, num_classes):
        super().__init__()
        self.features = nn.Sequential(
            nn.ReLU(inplace=True), nn.AvgPool2d(5, stride=3, padding=0, count_include_pad=False),
            nn.Conv2d(c, 128, 1, bias=False), nn.BatchNorm2d(128), nn.ReLU(inplace=True),
            nn.Conv2d(128, 768, 2, bias=False), nn.BatchNorm2d(768), nn.ReLU(inplace=True))
        self.classifier = nn.Linear(768, num_classes)

    def forward(self, x):
        return self.classifier(self.features(x).flatten(1))


class NetworkCIFAR(nn.Module):
    def __init__(self, C=36, num_classes=10, layers=20, auxiliary=True, genotype="FedNAS_V1"):
        super().__init__()
        genotype = genotypes.get(genotype)
        self.genotype_used = genotype
        self._layers = layers
        self._auxiliary = bool(auxiliary)
        self.drop_path_prob = 0.5
        cc = 3 * C
        self.stem = nn.Sequential(nn.Conv2d(3, cc, 3, padding=1, bias=False), nn.BatchNorm2d(cc))
        c_pp, c_p, c = cc, cc, C
        cells, red_prev, c_aux = [], False, None
        for i in range(layers):
            red = i in (layers // 3, 2 * layers // 3)
            if red:
                c *= 2
            cell = EvalCell(genotype, c_pp, c_p, c, red, red_prev)
            red_prev = red
            cells.append(cell)
            c_pp, c_p = c_p, cell.multiplier * c
            if i == 2 * layers // 3:
                c_aux = c_p
        self.cells = nn.ModuleList(cells)
        if self._auxiliary:
            self.auxiliary_head = AuxiliaryHeadCIFAR(c_aux, num_classes)
        self.global_pooling = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Linear(c_p, num_classes)

    def forward(self, x):
        aux = None
        s0 = s1 = self.stem(x)
        for i, cell in enumerate(self.cells):
            s0, s1 = s1, cell(s0, s1, self.drop_path_prob)
            if i == 2 * self._layers // 3 and self._auxiliary and self.training:
                aux = self.auxiliary_head(s1)
        return self.classifier(self.global_pooling(s1).flatten(1)), aux
