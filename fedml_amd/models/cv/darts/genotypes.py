"""DARTS search space and published cells (reference ``model/cv/darts/genotypes.py``).

A genotype lists, per cell type, two (operation, input-state) pairs for each intermediate node and the
states concatenated into the cell output."""
from collections import namedtuple

Genotype = namedtuple("Genotype", "normal normal_concat reduce reduce_concat")

# the 8 candidate operations of the search space (reference genotypes.py:5-14)
PRIMITIVES = ["none", "max_pool_3x3", "avg_pool_3x3", "skip_connect", "sep_conv_3x3", "sep_conv_5x5",
              "dil_conv_3x3", "dil_conv_5x5"]

# the second-order DARTS CIFAR-10 cell (Liu et al., 2019)
DARTS_V2 = Genotype(
    normal=[("sep_conv_3x3", 0), ("sep_conv_3x3", 1), ("sep_conv_3x3", 0), ("sep_conv_3x3", 1),
            ("sep_conv_3x3", 1), ("skip_connect", 0), ("skip_connect", 0), ("dil_conv_3x3", 2)],
    normal_concat=[2, 3, 4, 5],
    reduce=[("max_pool_3x3", 0), ("max_pool_3x3", 1), ("skip_connect", 2), ("max_pool_3x3", 1),
            ("max_pool_3x3", 0), ("skip_connect", 2), ("skip_connect", 2), ("max_pool_3x3", 1)],
    reduce_concat=[2, 3, 4, 5])
DARTS = DARTS_V2

# the cell FedNAS found on non-IID CIFAR-10 (the reference's `stage: train` default)
FedNAS_V1 = Genotype(
    normal=[("sep_conv_3x3", 1), ("sep_conv_3x3", 0), ("sep_conv_3x3", 2), ("sep_conv_5x5", 0),
            ("sep_conv_3x3", 1), ("sep_conv_5x5", 3), ("dil_conv_5x5", 3), ("sep_conv_3x3", 4)],
    normal_concat=[2, 3, 4, 5],
    reduce=[("max_pool_3x3", 0), ("skip_connect", 1), ("max_pool_3x3", 0), ("max_pool_3x3", 2),
            ("max_pool_3x3", 0), ("dil_conv_5x5", 1), ("max_pool_3x3", 0), ("dil_conv_5x5", 2)],
    reduce_concat=[2, 3, 4, 5])


def get(name) -> Genotype:
    """A genotype by name (``args.arch``), or a Genotype passed through."""
    if isinstance(name, Genotype):
        return name
    g = globals().get(str(name))
    if not isinstance(g, Genotype):
        raise KeyError(f"unknown DARTS genotype {name!r}")
    return g


def parse_alphas(weights, steps: int, cnn_from: int = 4):
    """Derive a cell from softmaxed architecture weights [edges, ops] (rows: node i's 2 + i input edges):
    per node keep the two strongest incoming edges (by their best non-'none' op) and that op. Returns
    (gene, count of picked ops whose index ≥ ``cnn_from``, the conv primitives)."""
    none = PRIMITIVES.index("none")
    gene, start, n, cnn = [], 0, 2, 0
    for i in range(steps):
        W = weights[start:start + n]
        edges = sorted(range(i + 2), key=lambda x: -max(W[x][k] for k in range(len(W[x])) if k != none))[:2]
        for j in edges:
            kb = max((k for k in range(len(W[j])) if k != none), key=lambda k: W[j][k])
            cnn += kb >= cnn_from
            gene.append((PRIMITIVES[kb], j))
        start += n
        n += 1
    return gene, cnn
