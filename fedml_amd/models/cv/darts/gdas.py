"""GDAS search network (reference ``model/cv/darts/model_search_gdas.py``): the same cells as DARTS, but
each edge samples ONE operation per forward pass — hard Gumbel-softmax over α with temperature τ
(straight-through gradient to α) — so only the sampled op runs instead of all eight."""
import torch
import torch.nn.functional as F

from .genotypes import Genotype, parse_alphas
from .search import Cell, MixedOp, Network


class GumbelMixedOp(MixedOp):
    def forward(self, x, w, active=None):
        """``active``: host-side indices of the non-zero entries of the one-hot ``w`` (only those ops run;
        multiplying by w[k] = 1 keeps the straight-through gradient path to α)."""
        ks = active if active is not None else [k for k in range(len(self._ops))]
        out = [w[k] * self._ops[k](x) for k in ks]
        return out[0] if len(out) == 1 else sum(out)


class GumbelCell(Cell):
    def __init__(self, *a):
        super().__init__(*a, mixed=GumbelMixedOp)

    def forward(self, s0, s1, weights):
        # ONE device→host read of the sampled one-hot weights per cell (the reference reads them per edge)
        picks = [[int(k) for k in torch.nonzero(row.detach().abs() > 1e-10).flatten().tolist()]
                 for row in weights.detach().cpu()]
        return self.edges([self.preprocess0(s0), self.preprocess1(s1)], weights,
                          lambda op, h, e: op(h, weights[e], picks[e]))


class Network_GumbelSoftmax(Network):
    def __init__(self, C=16, num_classes=10, layers=8, criterion=None, steps=4, multiplier=4, stem_multiplier=3,
                 tau=5.0):
        super().__init__(C, num_classes, layers, criterion, steps, multiplier, stem_multiplier)
        self.tau = float(tau)

    def _cell(self, *a):
        return GumbelCell(*a)

    def set_tau(self, tau):
        self.tau = float(tau)

    def get_tau(self):
        return self.tau

    def cell_weights(self, cell):
        return F.gumbel_softmax(self.alphas_reduce if cell.reduction else self.alphas_normal, self.tau, True)

    def genotype(self):
        """(genotype, #conv primitives in the normal cell, #conv primitives in the reduction cell)."""
        concat = list(range(2 + self._steps - self._multiplier, self._steps + 2))
        with torch.no_grad():
            normal, cn = parse_alphas(F.softmax(self.alphas_normal, -1).tolist(), self._steps)
            reduce, cr = parse_alphas(F.softmax(self.alphas_reduce, -1).tolist(), self._steps)
        return Genotype(normal, concat, reduce, concat), cn, cr
