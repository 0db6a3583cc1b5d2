"""FedNAS over message passing (reference: `mpi_p2p_mp/fednas/*`): clients run DARTS search
(weights + architecture alphas) on their shard; the server averages both and records the
derived genotype each round. ``args.stage`` = ``search`` | ``train``."""
import logging

from ...trainers.nas import ModelTrainerNAS
from .fl_protocol import FedAVGAggregator, run_fl


class FedNASAggregator(FedAVGAggregator):
    def aggregate(self):
        averaged = super().aggregate()
        model = self.trainer.model
        if hasattr(model, "genotype"):
            g = model.genotype()
            self.genotypes = getattr(self, "genotypes", []) + [g]
            logging.info("FedNAS genotype: %s", g)
        return averaged


def FedML_FedNAS_distributed(args, process_id, worker_number, comm, device, dataset, model, model_trainer=None,
                             preprocessed_sampling_lists=None):
    if model_trainer is None or not isinstance(model_trainer, ModelTrainerNAS):
        model_trainer = ModelTrainerNAS(model, args)
    out = run_fl(args, process_id, worker_number, comm, device, dataset, model, model_trainer,
                 aggregator_cls=FedNASAggregator, preprocessed_sampling_lists=preprocessed_sampling_lists)
    if out is not None:
        out["genotype"] = model_trainer.model.genotype()
    return out
