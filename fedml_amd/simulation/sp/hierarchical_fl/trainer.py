"""Hierarchical FL, sequential (reference: `single_process/hierarchical_fl/{trainer,group,client}.py`).

Clients are assigned to ``group_num`` groups (``group_method: random`` → ``np.random.randint``).
Each global round samples clients, every group runs ``group_comm_round`` rounds of FedAvg among
its sampled clients starting from the global model, and the server averages the groups
(weighted by their sampled sample counts). Like the reference, clients snapshot their model after
every local epoch and aggregation happens per *global epoch index*
(``(g·R_group + r)·E + e``), so the final global model after the last epoch is what a
centralised run over the same schedule would produce when there is one group and one client.
The reference's version is broken in this fork (it calls renamed FedAvg methods).
"""
import copy
import logging

import numpy as np

from ..fedavg.fedavg_api import FedAvgAPI


class HierarchicalTrainer(FedAvgAPI):
    def __init__(self, args, device, dataset, model, model_trainer=None):
        super().__init__(args, device, dataset, model, model_trainer)
        method = str(getattr(args, "group_method", "random"))
        if method != "random":
            raise ValueError(f"group_method {method} not supported (reference supports 'random')")
        self.group_num = int(getattr(args, "group_num", 1))
        self.group_indexes = np.random.randint(0, self.group_num, int(args.client_num_in_total))
        self.group_to_clients = {}
        for c, g in enumerate(self.group_indexes):
            self.group_to_clients.setdefault(int(g), []).append(c)
        self.global_rounds = int(getattr(args, "global_comm_round", getattr(args, "comm_round", 1)))
        self.group_rounds = int(getattr(args, "group_comm_round", 1))
        self.history = []

    def group_client_sampling(self, global_round_idx):
        sampled = self._client_sampling(global_round_idx, int(self.args.client_num_in_total),
                                        int(self.args.client_num_per_round))
        out = {}
        for c in sampled:
            out.setdefault(int(self.group_indexes[c]), []).append(int(c))
        return out

    def _client_epochs(self, cid, w, global_round_idx, group_round_idx):
        """Train client ``cid`` for ``epochs`` local epochs from w; snapshot after each epoch."""
        E = int(self.args.epochs)
        args1 = copy.copy(self.args)
        args1.epochs = 1
        self.model_trainer.set_id(cid)
        self.model_trainer.set_model_params(copy.deepcopy(w))
        snaps = []
        for e in range(E):
            self.model_trainer.train(self.train_data_local_dict[cid], self.device, args1)
            ge = (global_round_idx * self.group_rounds + group_round_idx) * E + e
            snaps.append((ge, self.model_trainer.get_model_params()))
        return snaps

    def _group_train(self, g, global_round_idx, w, clients):
        w_group, out = w, []
        for r in range(self.group_rounds):
            per_epoch = {}
            for c in clients:
                for ge, wl in self._client_epochs(c, w_group, global_round_idx, r):
                    per_epoch.setdefault(ge, []).append((self.train_data_local_num_dict[c], wl))
            for ge in sorted(per_epoch):
                out.append((ge, self._aggregate(per_epoch[ge])))
            w_group = out[-1][1]
        return out

    def train(self):
        w_global = self.model_trainer.get_model_params()
        freq = int(getattr(self.args, "frequency_of_the_test", 1) or 1)
        last_epoch = self.global_rounds * self.group_rounds * int(self.args.epochs) - 1
        for gr in range(self.global_rounds):
            groups = self.group_client_sampling(gr)
            by_epoch = {}
            for g in sorted(groups):
                n_g = sum(self.train_data_local_num_dict[c] for c in groups[g])
                for ge, wg in self._group_train(g, gr, w_global, groups[g]):
                    by_epoch.setdefault(ge, []).append((n_g, wg))
            for ge in sorted(by_epoch):
                w_global = self._aggregate(by_epoch[ge])
                if ge % freq == 0 or ge == last_epoch:
                    self.model_trainer.set_model_params(w_global)
                    stats = self._local_test_on_all_clients(ge)
                    stats["global_epoch"] = ge
                    self.history.append(stats)
            self.model_trainer.set_model_params(w_global)
        return w_global
