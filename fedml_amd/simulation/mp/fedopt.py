"""FedOpt, message-passing (reference: `mpi_p2p_mp/fedopt/FedOptAggregator.py:14-242`).

After FedAvg averaging the server treats ``w_global − avg`` as a pseudo-gradient and steps a
server optimizer (any torch optimizer by name — OptRepo). Optimizer state persists across
rounds (the reference re-instantiates it every round and copies the state back)."""
import torch

from ...core.arena import fedavg_state_dicts
from ..optrepo import server_optimizer
from .fl_protocol import FedAVGAggregator, run_fl


class FedOptAggregator(FedAVGAggregator):
    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.model = self.trainer.model
        self.opt = server_optimizer([p for p in self.model.parameters() if p.requires_grad], self.args)

    def aggregate(self):
        avg = fedavg_state_dicts(self._w_locals())
        params = dict(self.model.named_parameters())
        self.opt.zero_grad()
        with torch.no_grad():
            for name, p in params.items():
                p.grad = (p.data - avg[name].to(p.device, p.dtype)).clone()
        self.opt.step()
        # non-trainable buffers (BN stats) take the plain average
        sd = self.model.state_dict()
        with torch.no_grad():
            for k, v in sd.items():
                if k not in params:
                    v.copy_(avg[k].to(v.device, v.dtype))
        return self.get_global_model_params()


def FedML_FedOpt_distributed(args, process_id, worker_number, comm, device, dataset, model, model_trainer=None,
                             preprocessed_sampling_lists=None):
    return run_fl(args, process_id, worker_number, comm, device, dataset, model, model_trainer,
                  aggregator_cls=FedOptAggregator, preprocessed_sampling_lists=preprocessed_sampling_lists)
