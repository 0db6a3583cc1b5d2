"""Asymmetric (directed) topology (reference: `core/distributed/topology/asymmetric_topology_manager.py:7-110`).

Start from ring ∪ k-lattice with self loops; for every row, each zero entry is
turned into an out-link with probability 1/2 (``np.random.randint(2)`` draws,
same call sequence) unless the reverse link was already added; rows are then
normalised."""
import numpy as np

from .base_topology_manager import BaseTopologyManager, ring_lattice


class AsymmetricTopologyManager(BaseTopologyManager):
    def __init__(self, n, undirected_neighbor_num=3, out_directed_neighbor=3):
        self.n = n
        self.undirected_neighbor_num = undirected_neighbor_num
        self.out_directed_neighbor = out_directed_neighbor
        self.topology = []

    def generate_topology(self):
        n = self.n
        topo = np.maximum(ring_lattice(n, 2), ring_lattice(n, int(self.undirected_neighbor_num)))
        np.fill_diagonal(topo, 1.0)
        added = set()
        for i in range(n):
            zeros = [j for j in range(n) if topo[i, j] == 0]
            draws = np.random.randint(2, size=len(zeros))
            for d, j in zip(draws, zeros):
                if d == 1 and (j * n + i) not in added:
                    topo[i, j] = 1.0
                    added.add(i * n + j)
        self.topology = topo / topo.sum(axis=1, keepdims=True)

    def get_in_neighbor_weights(self, node_index):
        if node_index >= self.n:
            return []
        return [self.topology[r][node_index] for r in range(len(self.topology))]

    def get_out_neighbor_weights(self, node_index):
        return [] if node_index >= self.n else self.topology[node_index]

    def get_in_neighbor_idx_list(self, node_index):
        w = self.get_in_neighbor_weights(node_index)
        return [i for i, v in enumerate(w) if v > 0 and i != node_index]

    def get_out_neighbor_idx_list(self, node_index):
        w = self.get_out_neighbor_weights(node_index)
        return [i for i, v in enumerate(w) if v > 0 and i != node_index]
