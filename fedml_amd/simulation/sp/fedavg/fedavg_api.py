"""Sequential single-process FedAvg (Parrot SP; reference: `single_process/fedavg/fedavg_api.py:17-370`).

Behaviour kept: one shared trainer/model object for all simulated clients,
reference client sampling, sample-count weighted averaging of *every*
state_dict entry (BN buffers and counters included), periodic local tests on
all clients, global validation with accuracy + recall of ``target_label`` (fork).
Differences: accepts the standard 8-tuple *or* the fork's 9-tuple (Appendix A #4),
aggregation runs on the flat arena through the FedAvg kernel and does not mutate
the clients' dicts (Appendix A #10), results go to JSON instead of a pickle.
"""
import copy
import logging
import time

import torch

from ...common import client_sampling, fork_local_test_stats, log_metrics, save_results
from ....core.arena import fedavg_state_dicts
from ....trainers import create_model_trainer
from .client import Client


def unpack_dataset(dataset):
    if len(dataset) >= 9:
        return list(dataset[:8]) + [dataset[8]]
    return list(dataset) + [None]


class FedAvgAPI:
    def __init__(self, args, device, dataset, model, model_trainer=None):
        self.device = device
        self.args = args
        (train_num, test_num, train_global, test_global, num_dict, train_local, test_local, class_num,
         target_label) = unpack_dataset(dataset)
        self.train_global = train_global
        self.test_global = test_global
        self.val_global = None
        self.train_data_num_in_total = train_num
        self.test_data_num_in_total = test_num
        self.class_num = class_num
        self.target_label = target_label if target_label is not None else getattr(args, "target_label", None)
        self.train_data_local_num_dict = num_dict
        self.train_data_local_dict = train_local
        self.test_data_local_dict = test_local
        self.model_trainer = model_trainer or create_model_trainer(model, args)
        self.client_list = []
        self.res_dict = {}
        self._setup_clients()

    def _setup_clients(self):
        for client_idx in range(int(self.args.client_num_per_round)):
            self.client_list.append(Client(client_idx, self.train_data_local_dict[client_idx],
                                           self.test_data_local_dict[client_idx],
                                           self.train_data_local_num_dict[client_idx], self.args, self.device,
                                           self.model_trainer))

    def _client_sampling(self, round_idx, client_num_in_total, client_num_per_round):
        return client_sampling(round_idx, client_num_in_total, client_num_per_round)

    # public alias (reference hierarchical FL calls the un-prefixed names, Appendix A #9)
    client_sampling = _client_sampling

    def _aggregate(self, w_locals):
        return fedavg_state_dicts(w_locals)

    aggregate = _aggregate

    def train(self):
        w_global = self.model_trainer.get_model_params()
        freq = int(getattr(self.args, "frequency_of_the_test", 0) or 0)
        for round_idx in range(int(self.args.comm_round)):
            t0 = time.time()
            logging.info("################ Communication round : %d", round_idx)
            idxs = self._client_sampling(round_idx, int(self.args.client_num_in_total),
                                         int(self.args.client_num_per_round))
            w_locals = []
            for idx, client in enumerate(self.client_list):
                cid = idxs[idx]
                client.update_local_dataset(cid, self.train_data_local_dict[cid], self.test_data_local_dict[cid],
                                            self.train_data_local_num_dict[cid])
                w = client.train(copy.deepcopy(w_global))
                w_locals.append((client.get_sample_number(), w))
            w_global = self._aggregate(w_locals)
            self.model_trainer.set_model_params(w_global)
            rec = self.res_dict.setdefault(round_idx, {})
            last = round_idx == int(self.args.comm_round) - 1
            if last or (freq > 0 and round_idx % freq == 0):
                rec.update(self._local_test_on_all_clients(round_idx))
            if last or (freq > 0 and round_idx % freq == 0):
                acc, recall = self._validate_global_model(self.model_trainer.model, self.test_global, self.device)
                rec["Global/Acc"], rec["Global/Recall"] = acc, recall
                rec["Global/Loss"] = self._last_global_loss
            rec["round_time_s"] = time.time() - t0
        out = getattr(self.args, "results_path", None)
        if out:
            save_results(self.res_dict, out)
        return w_global

    def _local_test_on_all_clients(self, round_idx):
        train_m, test_m = [], []
        for cid in range(int(self.args.client_num_in_total)):
            if self.test_data_local_dict.get(cid) is None:
                continue
            client = self.client_list[0]
            client.update_local_dataset(cid, self.train_data_local_dict[cid], self.test_data_local_dict[cid],
                                        self.train_data_local_num_dict[cid])
            train_m.append(client.local_test(False))
            test_m.append(client.local_test(True))
        stats = fork_local_test_stats(train_m, test_m)
        log_metrics(stats, round_idx)
        return stats

    def _validate_global_model(self, model, data, device):
        m = self.model_trainer.test(data, device, self.args)
        acc = m["test_correct"] / max(1, m["test_total"])
        self._last_global_loss = m["test_loss"] / max(1, m["test_total"])
        recall = None
        if self.target_label is not None and "recall_per_class" in m:
            recall = m["recall_per_class"][int(self.target_label)]
        return acc, recall
