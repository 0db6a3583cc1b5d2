"""FedAvg with robust aggregation, sequential (reference: `single_process/fedavg_robust/*`):
backdoor attacker at ``attacker_index`` every ``attack_freq`` rounds; norm-diff clipping /
weak DP / coordinate median defenses; reports main and targeted-task accuracy."""
import copy

from ....core.robustness import RobustAggregator
from ....core.server_update import robust_aggregate
from ....data.backdoor import backdoor_test_set, poison_client_data
from ....data.client_data import concat_client_data
from ..fedavg.fedavg_api import FedAvgAPI


class FedAvgRobustAPI(FedAvgAPI):
    def __init__(self, args, device, dataset, model, model_trainer=None):
        super().__init__(args, device, dataset, model, model_trainer)
        self.robust = RobustAggregator(args)
        self._round = 0
        self._glob = None
        tgt = int(getattr(args, "backdoor_target", 0))
        tests = [v for v in self.test_data_local_dict.values() if v is not None]
        self.targeted_test = backdoor_test_set(concat_client_data(tests), tgt) if tests else None
        self.attacker_index = int(getattr(args, "attacker_index", 1))
        self.attack_freq = int(getattr(args, "attack_freq", 1) or 1)
        self.targeted_history = []
        for c in self.client_list:
            c._orig_train = c.train
            c.train = self._wrap(c)

    def _wrap(self, client):
        def train(w_global):
            self._glob = copy.deepcopy(w_global)
            if client.client_idx == self.attacker_index and self._round % self.attack_freq == 0:
                orig = client.local_training_data
                client.local_training_data = poison_client_data(orig, int(getattr(self.args, "backdoor_target", 0)))
                try:
                    return client._orig_train(w_global)
                finally:
                    client.local_training_data = orig
            return client._orig_train(w_global)
        return train

    def _aggregate(self, w_locals):
        avg = robust_aggregate(self.robust, w_locals, self._glob, self._round)
        self._round += 1
        if self.targeted_test is not None and self.targeted_test.num_samples:
            self.model_trainer.set_model_params(avg)
            m = self.model_trainer.test(self.targeted_test, self.device, self.args)
            self.targeted_history.append(m["test_correct"] / max(1, m["test_total"]))
        return avg

    aggregate = _aggregate
