"""FedOpt, message-passing (reference: `mpi_p2p_mp/fedopt/FedOptAggregator.py:14-242`).

After FedAvg averaging the server treats ``w_global − avg`` as a pseudo-gradient and steps a
server optimizer (any torch optimizer by name — OptRepo). Optimizer state persists across
rounds (the reference re-instantiates it every round and copies the state back)."""
from ...core.arena import fedavg_state_dicts
from ...core.server_update import ServerOptimizer
from .fl_protocol import FedAVGAggregator, run_fl


class FedOptAggregator(FedAVGAggregator):
    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.server_opt = ServerOptimizer(self.trainer.model, self.args)

    def aggregate(self):
        new = self.server_opt.apply(fedavg_state_dicts(self._w_locals()))
        self.set_global_model_params(new)
        return new


def FedML_FedOpt_distributed(args, process_id, worker_number, comm, device, dataset, model, model_trainer=None,
                             preprocessed_sampling_lists=None):
    return run_fl(args, process_id, worker_number, comm, device, dataset, model, model_trainer,
                  aggregator_cls=FedOptAggregator, preprocessed_sampling_lists=preprocessed_sampling_lists)
