"""Cross-silo federated learning: horizontal (one process per silo) and hierarchical (a Cheetah
data-parallel group of GPUs inside each silo) — reference `python/fedml/cross_silo/`."""
from .client import Client
from .server import Server
from . import hierarchical
