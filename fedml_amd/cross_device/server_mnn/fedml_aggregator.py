"""Cross-device aggregator over model FILES (reference: `cross_device/server_mnn/fedml_aggregator.py:16-222`).

Each uploaded device model is a file path; the server reads every file into an indexed tensor
dict (codec), averages them on the flat arena (FedAvg kernel on MI355X), writes the global model
file, and evaluates by loading the indexed tensors into the torch twin of the on-device model.
"""
import logging
import time

import numpy as np
import torch

from ...core.arena import fedavg_state_dicts
from ...simulation.common import summarize_metrics
from ..model_codec import get_codec, load_indexed, model_to_indexed


class FedMLAggregator:
    def __init__(self, test_global, all_train_data_num, train_data_local_num_dict, worker_num, device, args,
                 model_trainer):
        self.trainer = model_trainer
        self.args = args
        self.test_global = test_global
        self.all_train_data_num = all_train_data_num
        self.train_data_local_num_dict = train_data_local_num_dict
        self.worker_num = worker_num
        self.device = device
        self.codec = get_codec(args)
        self.global_model_file_path = getattr(args, "global_model_file_path", None) or "./model_file_cache/global_model" + \
            self.codec.suffix
        self.model_dict, self.sample_num_dict = {}, {}
        self.flag_client_model_uploaded_dict = {i: False for i in range(worker_num)}
        self.history = []
        # materialise the initial global model file from the torch twin
        self.codec.write(self.global_model_file_path, model_to_indexed(self.trainer.model))

    def get_global_model_params(self):
        return self.global_model_file_path

    def set_global_model_params(self, path):
        load_indexed(self.trainer.model, self.codec.read(path))

    def add_local_trained_result(self, index, model_file, sample_num):
        self.model_dict[index] = model_file
        self.sample_num_dict[index] = sample_num
        self.flag_client_model_uploaded_dict[index] = True

    def check_whether_all_receive(self):
        if not all(self.flag_client_model_uploaded_dict[i] for i in range(self.worker_num)):
            return False
        for i in range(self.worker_num):
            self.flag_client_model_uploaded_dict[i] = False
        return True

    def aggregate(self):
        t0 = time.time()
        w_locals = []
        for i in range(self.worker_num):
            d = self.codec.read(self.model_dict[i])
            w_locals.append((self.sample_num_dict[i], {str(k): v for k, v in d.items()}))
        avg = fedavg_state_dicts(w_locals)
        indexed = {int(k): v for k, v in avg.items()}
        self.codec.write(self.global_model_file_path, indexed, template_path=self.model_dict[0])
        load_indexed(self.trainer.model, indexed)
        logging.info("cross-device aggregate of %d device models: %.3f s", self.worker_num, time.time() - t0)
        return self.global_model_file_path

    def data_silo_selection(self, round_idx, data_silo_num_in_total, client_num_in_total):
        if data_silo_num_in_total == client_num_in_total:
            return list(range(data_silo_num_in_total))
        np.random.seed(round_idx)
        return np.random.choice(range(data_silo_num_in_total), client_num_in_total, replace=False).tolist()

    def client_selection(self, round_idx, client_id_list_in_total, client_num_per_round):
        if client_num_per_round == len(client_id_list_in_total):
            return list(client_id_list_in_total)
        np.random.seed(round_idx)
        return np.random.choice(client_id_list_in_total, client_num_per_round, replace=False).tolist()

    def test_on_server_for_all_clients(self, round_idx):
        if self.test_global is None:
            return None
        m = self.trainer.test(self.test_global, self.device, self.args)
        acc, loss = summarize_metrics([m])
        stats = {"round": round_idx, "Test/Acc": acc, "Test/Loss": loss}
        self.history.append(stats)
        logging.info("cross-device server test: %s", stats)
        return stats
