"""FedAvg-robust, message-passing (reference: `mpi_p2p_mp/fedavg_robust/*`).

Attack: worker holding client index ``attacker_index`` (default 1) trains on a backdoored copy of
its data every ``attack_freq`` rounds. Defenses (``defense_type``): ``norm_diff_clipping``
(clip each update's ‖Δ‖ to ``norm_bound``), ``weak_dp`` (clip + Gaussian noise ``stddev`` on the
aggregate), ``coordinate_median``. The server reports main-task accuracy and targeted-task
(backdoor) accuracy."""
import logging

import torch

from ...core.server_update import robust_aggregate
from ...core.robustness import RobustAggregator
from ...data.backdoor import backdoor_test_set, poison_client_data
from ...data.client_data import concat_client_data
from .fl_protocol import FedAVGAggregator, FedAVGTrainer, run_fl


class FedAvgRobustAggregator(FedAVGAggregator):
    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.robust = RobustAggregator(self.args)
        self.round = 0
        tgt = int(getattr(self.args, "backdoor_target", 0))
        self.targeted_test = backdoor_test_set(concat_client_data(list(self.test_data_local_dict.values())), tgt) \
            if self.test_data_local_dict else None

    def aggregate(self):
        avg = robust_aggregate(self.robust, self._w_locals(), self.get_global_model_params(), self.round)
        self.set_global_model_params(avg)
        self.round += 1
        return avg

    def test_on_server_for_all_clients(self, round_idx):
        stats = super().test_on_server_for_all_clients(round_idx)
        if stats is not None and self.targeted_test is not None and self.targeted_test.num_samples:
            m = self.trainer.test(self.targeted_test, self.device, self.args)
            stats["Targeted/Acc"] = m["test_correct"] / max(1, m["test_total"])
            logging.info("targeted-task accuracy: %.4f", stats["Targeted/Acc"])
        return stats


class FedAvgRobustTrainer(FedAVGTrainer):
    def train(self, round_idx=None):
        attacker = int(getattr(self.args, "attacker_index", 1))
        freq = int(getattr(self.args, "attack_freq", 0) or 0)
        data = self.train_local
        if freq > 0 and self.client_index == attacker and round_idx is not None and round_idx % freq == 0:
            data = poison_client_data(self.train_local, int(getattr(self.args, "backdoor_target", 0)))
            logging.info("client %d: backdoor attack in round %d", self.client_index, round_idx)
        self.args.round_idx = round_idx
        self.trainer.train(data, self.device, self.args)
        return self.trainer.get_model_params(), self.local_sample_number


def FedML_FedAvgRobust_distributed(args, process_id, worker_number, comm, device, dataset, model,
                                   model_trainer=None, preprocessed_sampling_lists=None):
    return run_fl(args, process_id, worker_number, comm, device, dataset, model, model_trainer,
                  aggregator_cls=FedAvgRobustAggregator, trainer_cls=FedAvgRobustTrainer,
                  preprocessed_sampling_lists=preprocessed_sampling_lists)
