"""Cross-silo server-side aggregator (reference: `cross_silo/horizontal/fedml_aggregator.py:13-263`).

Aggregation runs on the flat arena (``fedavg_state_dicts`` → FedAvg HIP kernel on MI355X) with no
list↔tensor conversion (the wire format carries raw tensors). An optional
``ServerAggregator`` (user hook, reference `core/alg_frame/server_aggregator.py`) owns the global
model and evaluation; by default the model trainer is used for both.
"""
import logging
import time

import numpy as np
import torch

from ...core.arena import fedavg_state_dicts
from ...core.mlops import MLOpsMetrics
from ...ops import weighted_sum
from ...simulation.common import client_sampling, summarize_metrics


class FedMLAggregator:
    def __init__(self, train_global, test_global, all_train_data_num, train_data_local_dict, test_data_local_dict,
                 train_data_local_num_dict, client_num, device, args, server_aggregator):
        self.aggregator = server_aggregator
        self.trainer = server_aggregator  # reference attribute name
        self.args = args
        self.train_global, self.test_global = train_global, test_global
        self.val_global = None
        self.all_train_data_num = all_train_data_num
        self.train_data_local_dict = train_data_local_dict
        self.test_data_local_dict = test_data_local_dict
        self.train_data_local_num_dict = train_data_local_num_dict
        self.client_num = client_num
        self.device = device
        self.model_dict, self.sample_num_dict = {}, {}
        self.flag_client_model_uploaded_dict = {i: False for i in range(client_num)}
        self.history = []
        self.flat_layout = None      # set by the server manager on the same-node device plane
        self._flat_global = None     # newest aggregate as a flat device tensor (state dict made lazily)

    def get_global_model_params(self):
        if self._flat_global is not None:
            self.aggregator.set_model_params(self.flat_layout.unflatten(self._flat_global))
            self._flat_global = None
        return self.aggregator.get_model_params()

    def set_global_model_params(self, model_parameters):
        self._flat_global = None
        self.aggregator.set_model_params(model_parameters)

    def add_local_trained_result(self, index, model_params, sample_num):
        self.model_dict[index] = model_params
        self.sample_num_dict[index] = sample_num
        self.flag_client_model_uploaded_dict[index] = True

    def check_whether_all_receive(self):
        if not all(self.flag_client_model_uploaded_dict.values()):
            return False
        for i in self.flag_client_model_uploaded_dict:
            self.flag_client_model_uploaded_dict[i] = False
        return True

    def aggregate(self):
        t0 = time.time()
        hooked = callable(getattr(self.aggregator, "on_before_aggregation", None)) or \
            callable(getattr(self.aggregator, "on_after_aggregation", None))
        if hooked and self.model_dict and all(torch.is_tensor(v) for v in self.model_dict.values()):
            # a user aggregator with aggregation hooks (robust aggregation, DP noise) sees state dicts on the
            # device plane too: the flat slot rows are unflattened (device-side views, no host copy)
            for i in list(self.model_dict):
                self.model_dict[i] = self.flat_layout.unflatten(self.model_dict[i], clone=False)
        if self.model_dict and all(torch.is_tensor(v) for v in self.model_dict.values()):
            # flat device uploads (device mailbox slots): one FedAvg kernel over the stacked rows; the
            # result stays a flat device tensor (the state-dict hooks do not apply on this plane)
            idx = sorted(self.model_dict)
            counts = [float(self.sample_num_dict[i]) for i in idx]
            stack = torch.stack([self.model_dict[i] for i in idx])
            w = torch.tensor([c / sum(counts) for c in counts], dtype=torch.float32, device=stack.device)
            avg = weighted_sum(stack, w)
            self._flat_global = avg
            self.model_dict.clear()
            self.sample_num_dict.clear()
            logging.info("aggregate (device plane) time cost: %.3f s", time.time() - t0)
            return avg
        w_locals = [(self.sample_num_dict[i], self.model_dict[i]) for i in sorted(self.model_dict)]
        hook = getattr(self.aggregator, "on_before_aggregation", None)
        if callable(hook):
            w_locals = hook(w_locals)
        avg = fedavg_state_dicts(w_locals)
        hook = getattr(self.aggregator, "on_after_aggregation", None)
        if callable(hook):
            avg = hook(avg)
        self.set_global_model_params(avg)
        self.model_dict.clear()
        self.sample_num_dict.clear()
        logging.info("aggregate time cost: %.3f s", time.time() - t0)
        return avg

    def data_silo_selection(self, round_idx, client_num_in_total, client_num_per_round):
        assert client_num_in_total >= client_num_per_round
        np.random.seed(round_idx)
        return np.random.choice(range(client_num_in_total), client_num_per_round, replace=False).tolist()

    def client_selection(self, round_idx, client_id_list_in_total, client_num_per_round):
        if client_num_per_round == len(client_id_list_in_total):
            return list(client_id_list_in_total)
        np.random.seed(round_idx)
        return np.random.choice(client_id_list_in_total, client_num_per_round, replace=False).tolist()

    def client_sampling(self, round_idx, client_num_in_total, client_num_per_round):
        return client_sampling(round_idx, client_num_in_total, client_num_per_round)

    def test_on_server_for_all_clients(self, round_idx):
        freq = int(getattr(self.args, "frequency_of_the_test", 0) or 0)
        last = round_idx == int(self.args.comm_round) - 1
        if not (last or (freq > 0 and round_idx % freq == 0)):
            return None
        if self.aggregator.test_on_the_server(self.train_data_local_dict, self.test_data_local_dict, self.device,
                                              self.args):
            return None
        if self.test_global is None:
            return None
        if self._flat_global is not None:   # device-plane aggregate: materialise the model for the test
            self.get_global_model_params()
        m = self.aggregator.test(self.test_global, self.device, self.args)
        acc, loss = summarize_metrics([m])
        stats = {"round": round_idx, "Test/Acc": acc, "Test/Loss": loss}
        self.history.append(stats)
        MLOpsMetrics.get_instance().log(stats, step=round_idx)
        logging.info("cross-silo server test: %s", stats)
        return stats
