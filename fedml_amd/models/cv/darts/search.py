"""DARTS search network for FedNAS (reference ``model/cv/darts/model_search.py``).

Every edge of a cell is a MixedOp: the softmax(α)-weighted sum of all 8 candidate operations
(``genotypes.PRIMITIVES``); normal and reduction cells share one α matrix each. ``arch_parameters()`` /
``weight_parameters()`` / ``new()`` / ``genotype()`` are the interface FedNAS' trainer and aggregator use
(``mpi_p2p_mp/fednas/FedNASTrainer.py``); the α live in the state dict, so the FedAvg aggregator averages
weights and architecture together."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .genotypes import PRIMITIVES, Genotype, parse_alphas
from .operations import OPS, FactorizedReduce, ReLUConvBN


class MixedOp(nn.Module):
    def __init__(self, c, stride):
        super().__init__()
        ops = []
        for p in PRIMITIVES:
            op = OPS[p](c, stride, False)
            if "pool" in p:   # pooled features are re-normalised before mixing
                op = nn.Sequential(op, nn.BatchNorm2d(c, affine=False))
            ops.append(op)
        self._ops = nn.ModuleList(ops)

    def forward(self, x, w):
        return sum(wi * op(x) for wi, op in zip(w, self._ops))


class Cell(nn.Module):
    def __init__(self, steps, multiplier, c_pp, c_p, c, reduction, reduction_prev, mixed=MixedOp):
        super().__init__()
        self.reduction = reduction
        self.preprocess0 = FactorizedReduce(c_pp, c, affine=False) if reduction_prev else \
            ReLUConvBN(c_pp, c, 1, 1, 0, affine=False)
        self.preprocess1 = ReLUConvBN(c_p, c, 1, 1, 0, affine=False)
        self._steps, self._multiplier = steps, multiplier
        self._ops = nn.ModuleList(mixed(c, 2 if reduction and j < 2 else 1) for i in range(steps) for j in range(2 + i))

    def edges(self, states, weights, edge_fn):
        off = 0
        for _ in range(self._steps):
            s = sum(edge_fn(self._ops[off + j], h, off + j) for j, h in enumerate(states))
            off += len(states)
            states.append(s)
        return torch.cat(states[-self._multiplier:], 1)

    def forward(self, s0, s1, weights):
        return self.edges([self.preprocess0(s0), self.preprocess1(s1)], weights,
                          lambda op, h, e: op(h, weights[e]))


class Network(nn.Module):
    """``Network(C, num_classes, layers, criterion=None, steps=4, multiplier=4, stem_multiplier=3)``: the
    reference's search network (cells at layers//3 and 2·layers//3 reduce)."""

    def __init__(self, C=16, num_classes=10, layers=8, criterion=None, steps=4, multiplier=4, stem_multiplier=3):
        super().__init__()
        self._C, self._num_classes, self._layers = C, num_classes, layers
        self._steps, self._multiplier, self._stem_multiplier = steps, multiplier, stem_multiplier
        self._criterion = criterion or nn.CrossEntropyLoss()
        cc = stem_multiplier * C
        self.stem = nn.Sequential(nn.Conv2d(3, cc, 3, padding=1, bias=False), nn.BatchNorm2d(cc))
        c_pp, c_p, c = cc, cc, C
        cells, red_prev = [], False
        for i in range(layers):
            red = i in (layers // 3, 2 * layers // 3)
            if red:
                c *= 2
            cells.append(self._cell(steps, multiplier, c_pp, c_p, c, red, red_prev))
            red_prev = red
            c_pp, c_p = c_p, multiplier * c
        self.cells = nn.ModuleList(cells)
        self.global_pooling = nn.AdaptiveAvgPool2d(1)
        self.classifier = nn.Linear(c_p, num_classes)
        k = sum(2 + i for i in range(steps))
        self.alphas_normal = nn.Parameter(1e-3 * torch.randn(k, len(PRIMITIVES)))
        self.alphas_reduce = nn.Parameter(1e-3 * torch.randn(k, len(PRIMITIVES)))

    def _cell(self, *a):
        return Cell(*a)

    def arch_parameters(self):
        return [self.alphas_normal, self.alphas_reduce]

    def weight_parameters(self):
        ids = {id(p) for p in self.arch_parameters()}
        return [p for p in self.parameters() if id(p) not in ids]

    def _ctor_args(self):
        return dict(C=self._C, num_classes=self._num_classes, layers=self._layers, criterion=self._criterion,
                    steps=self._steps, multiplier=self._multiplier, stem_multiplier=self._stem_multiplier)

    def new(self):
        m = type(self)(**self._ctor_args()).to(self.alphas_normal.device)
        for a, b in zip(m.arch_parameters(), self.arch_parameters()):
            a.data.copy_(b.data)
        return m

    def cell_weights(self, cell):
        return F.softmax(self.alphas_reduce if cell.reduction else self.alphas_normal, dim=-1)

    def forward(self, x):
        s0 = s1 = self.stem(x)
        for cell in self.cells:
            s0, s1 = s1, cell(s0, s1, self.cell_weights(cell))
        return self.classifier(self.global_pooling(s1).flatten(1))

    def _loss(self, x, y):
        return self._criterion(self(x), y)

    def genotype(self):
        concat = list(range(2 + self._steps - self._multiplier, self._steps + 2))
        with torch.no_grad():
            normal, _ = parse_alphas(F.softmax(self.alphas_normal, -1).tolist(), self._steps)
            reduce, _ = parse_alphas(F.softmax(self.alphas_reduce, -1).tolist(), self._steps)
        return Genotype(normal, concat, reduce, concat)
