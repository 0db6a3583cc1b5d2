"""DARTS / GDAS search spaces and the genotype-built evaluation network for FedNAS (reference
``model/cv/darts/*``): ``Network`` (DARTS search, continuous relaxation), ``Network_GumbelSoftmax``
(GDAS search, one sampled op per edge), ``NetworkCIFAR`` (``stage: train``)."""
from .eval_net import AuxiliaryHeadCIFAR, NetworkCIFAR, drop_path
from .gdas import Network_GumbelSoftmax
from .genotypes import DARTS, DARTS_V2, PRIMITIVES, FedNAS_V1, Genotype
from .operations import OPS
from .search import Cell, MixedOp, Network

__all__ = ["Network", "Network_GumbelSoftmax", "NetworkCIFAR", "AuxiliaryHeadCIFAR", "Cell", "MixedOp", "OPS",
           "PRIMITIVES", "Genotype", "DARTS", "DARTS_V2", "FedNAS_V1", "drop_path"]
