"""FedNova, sequential (reference: `single_process/fednova/fednova_trainer.py:12-295`): clients
run the FedNova optimizer (``trainers.fednova``); the server applies the normalised average
(+ optional global momentum ``gmf``) as one weighted sum over the client stack."""
import copy
import time

from ....core.server_update import fednova_aggregate
from ....trainers.fednova import ModelTrainerFedNova
from ..fedavg.fedavg_api import FedAvgAPI


class FedNovaAPI(FedAvgAPI):
    def __init__(self, args, device, dataset, model, model_trainer=None):
        super().__init__(args, device, dataset, model, model_trainer or ModelTrainerFedNova(model, args))
        self.momentum_buf = None

    def train(self):
        w_global = self.model_trainer.get_model_params()
        freq = int(getattr(self.args, "frequency_of_the_test", 0) or 0)
        for round_idx in range(int(self.args.comm_round)):
            t0 = time.time()
            idxs = self._client_sampling(round_idx, int(self.args.client_num_in_total),
                                         int(self.args.client_num_per_round))
            total = float(sum(self.train_data_local_num_dict[c] for c in idxs))
            w_locals, ratios, a_vec, taus = [], [], [], []
            for idx, client in enumerate(self.client_list):
                cid = idxs[idx]
                client.update_local_dataset(cid, self.train_data_local_dict[cid], self.test_data_local_dict[cid],
                                            self.train_data_local_num_dict[cid])
                ratio = self.train_data_local_num_dict[cid] / total
                self.model_trainer.set_model_params(copy.deepcopy(w_global))
                self.model_trainer.train(client.local_training_data, self.device, self.args, ratio=ratio)
                w_locals.append(self.model_trainer.get_model_params())
                ratios.append(ratio)
                a_vec.append(self.model_trainer.a_i)
                taus.append(self.model_trainer.tau_eff_i)
            # the reference starts every round with an empty global momentum buffer (fednova_trainer.py:80)
            if not bool(getattr(self.args, "fednova_gmf_persist", False)):
                self.momentum_buf = None
            w_global, self.momentum_buf = fednova_aggregate(
                w_global, w_locals, ratios, a_vec, taus, gmf=float(getattr(self.args, "gmf", 0.0) or 0.0),
                lr=float(self.args.learning_rate), momentum_buf=self.momentum_buf)
            self.model_trainer.set_model_params(w_global)
            rec = self.res_dict.setdefault(round_idx, {})
            if round_idx == int(self.args.comm_round) - 1 or (freq > 0 and round_idx % freq == 0):
                rec.update(self._local_test_on_all_clients(round_idx))
            rec["round_time_s"] = time.time() - t0
        return w_global
