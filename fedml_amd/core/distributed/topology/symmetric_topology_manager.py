"""Symmetric topology: ring ∪ k-regular lattice, self loops, row-normalised
(reference: `core/distributed/topology/symmetric_topology_manager.py:7-82`)."""
import numpy as np

from .base_topology_manager import BaseTopologyManager, ring_lattice


class SymmetricTopologyManager(BaseTopologyManager):
    def __init__(self, n, neighbor_num=2):
        self.n = n
        self.neighbor_num = neighbor_num
        self.topology = []

    def generate_topology(self):
        adj = np.maximum(ring_lattice(self.n, 2), ring_lattice(self.n, int(self.neighbor_num)))
        np.fill_diagonal(adj, 1.0)
        self.topology = adj / adj.sum(axis=1, keepdims=True)

    def get_in_neighbor_weights(self, node_index):
        return [] if node_index >= self.n else self.topology[node_index]

    def get_out_neighbor_weights(self, node_index):
        return [] if node_index >= self.n else self.topology[node_index]

    def get_in_neighbor_idx_list(self, node_index):
        w = self.get_in_neighbor_weights(node_index)
        return [i for i, v in enumerate(w) if v > 0 and i != node_index]

    def get_out_neighbor_idx_list(self, node_index):
        w = self.get_out_neighbor_weights(node_index)
        return [i for i, v in enumerate(w) if v > 0 and i != node_index]
