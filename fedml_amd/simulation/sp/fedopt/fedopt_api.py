"""FedOpt, sequential (reference: `single_process/fedopt/fedopt_api.py:13-299`): FedAvg followed
by a persistent server optimizer step on the pseudo-gradient (``core.server_update``)."""
from ....core.arena import fedavg_state_dicts
from ....core.server_update import ServerOptimizer
from ..fedavg.fedavg_api import FedAvgAPI


class FedOptAPI(FedAvgAPI):
    def __init__(self, args, device, dataset, model, model_trainer=None):
        super().__init__(args, device, dataset, model, model_trainer)
        self.server_opt = ServerOptimizer(self.model_trainer.model, args)

    def _aggregate(self, w_locals):
        return self.server_opt.apply(fedavg_state_dicts(w_locals))

    aggregate = _aggregate
