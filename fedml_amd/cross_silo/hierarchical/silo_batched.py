"""A silo that trains several LOCAL clients per round on the client-batched engine, data-parallel over
the silo's processes (BASELINE config 5: hierarchical cross-silo FedAvg, 8 silos × 4 local clients,
Cheetah DP inside each silo).

Reference roles (``cross_silo/hierarchical/client_master_manager.py:239-249``,
``trainer_dist_adapter.py:56-66,125``): the silo master receives the global model, the silo's
processes train together and the master uploads one model for the silo. Here a silo holds
``silo_local_clients`` clients (its data split into that many equal shards); every silo process
hosts a share of them in a ``ClientBatchEngine`` (one client stack per GPU, native HIP kernels /
batched transformer) and the silo's process group reduces Σ n_c·w_c ‖ Σ n_c in ONE flat all-reduce
(RCCL within the silo's GPUs — the same round as ``simulation.rccl.RCCLSimulator`` with the silo as
the world). The master uploads the silo's sample-weighted average with the silo's sample count, so
the server's FedAvg over silos equals FedAvg over all silos' clients (tested against the flat
simulator, ``tests/test_hier_silo.py``)."""
import copy
import logging

import torch

from ...data.client_data import ClientData
from ...parallel import comm
from ...simulation.rccl.client_store import DeviceClientStore


def split_local_clients(cd: ClientData, n: int):
    """The silo's samples as ``n`` contiguous equal shards (the last takes the remainder)."""
    N = len(cd.x)
    per = N // n
    offs = [i * per for i in range(n)]
    counts = [per] * (n - 1) + [N - per * (n - 1)]
    return offs, counts


class SiloBatchedTrainer:
    """Trains a silo's local clients; ``train(round_idx)`` leaves the silo average in ``model``."""

    def __init__(self, args, device, model, silo_data: ClientData, n_local: int):
        from ...simulation.rccl.simulator import RCCLSimulator
        self.args = args
        self.device = torch.device(device)
        self.n_local = int(n_local)
        self._stores = {}
        store, counts = self._store(None, silo_data)
        a = copy.copy(args)
        a.client_num_in_total = self.n_local
        a.client_num_per_round = self.n_local
        a.comm_round = 1
        a.frequency_of_the_test = 0
        a.checkpoint_dir = None
        a.federated_optimizer = "FedAvg"   # the SERVER runs the federated optimizer over silos
        self.sim = RCCLSimulator(a, self.device, None, model, store=store)
        self.num_samples = int(sum(counts))
        self.last_loss = None
        logging.info("silo: %d local clients (%s samples), %d of them on this process", self.n_local, counts,
                     len(self.sim.assignment(0)[1]))

    def _store(self, key, silo_data: ClientData):
        offs, counts = split_local_clients(silo_data, self.n_local)
        st = DeviceClientStore(silo_data.x.to(self.device), silo_data.y.to(self.device), offs, counts)
        self._stores[key] = st
        return st, counts

    def set_data(self, key, silo_data: ClientData):
        """Train on another data shard from now on (the server assigns silos a data index per round): the
        engine, its arenas and its captured graphs are kept — only the device data store changes (cached per
        index)."""
        st = self._stores.get(key)
        if st is None:
            st, _ = self._store(key, silo_data)
        self.sim.store = st
        self.sim.sample_counts = st.counts_host
        self.num_samples = int(sum(st.counts_host))

    def load_global(self, params):
        """A state dict, or the flat global model (device tensor, e.g. the device plane's shared buffer)."""
        if torch.is_tensor(params):
            self.sim.global_flat.copy_(params.reshape(-1))
            return
        self.sim.global_flat.copy_(self.sim.layout.flatten(params, device=self.device))

    def sync(self):
        """Collective over the silo: every process leaves with the master's global model."""
        comm.broadcast_flat(self.sim.global_flat, 0)

    def train(self, round_idx: int):
        self.sim.run_round(int(round_idx))
        self.last_loss = self.sim.engine.last_loss
        return self.sim.global_model_state()
