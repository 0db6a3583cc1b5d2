"""Topology manager interface (reference: `core/distributed/topology/base_topology_manager.py:4-23`)."""
import abc

import numpy as np


def ring_lattice(n: int, k: int) -> np.ndarray:
    """Adjacency of a Watts–Strogatz graph with rewiring p=0: each node joined to its
    k//2 nearest neighbours on each side (what `nx.watts_strogatz_graph(n, k, 0)` builds).
    networkx is not required."""
    a = np.zeros((n, n), dtype=np.float32)
    half = k // 2
    for i in range(n):
        for d in range(1, half + 1):
            j = (i + d) % n
            if j != i:
                a[i, j] = 1.0
                a[j, i] = 1.0
    return a


class BaseTopologyManager(abc.ABC):
    topology: np.ndarray

    @abc.abstractmethod
    def generate_topology(self):
        pass

    @abc.abstractmethod
    def get_in_neighbor_idx_list(self, node_index):
        pass

    @abc.abstractmethod
    def get_out_neighbor_idx_list(self, node_index):
        pass

    @abc.abstractmethod
    def get_in_neighbor_weights(self, node_index):
        pass

    @abc.abstractmethod
    def get_out_neighbor_weights(self, node_index):
        pass

    def mixing_matrix(self, device=None):
        """Row-stochastic mixing matrix as a torch tensor (for batched gossip = W @ X)."""
        import torch
        return torch.as_tensor(np.asarray(self.topology, dtype=np.float32), device=device)
