"""FedNAS over message passing (reference: `mpi_p2p_mp/fednas/*`). ``args.stage``:

* ``search`` — clients run DARTS (or GDAS) search (weights + architecture alphas) on their shard; the
  server averages both (FedNASAggregator.__aggregate_weight / __aggregate_alpha) and records the derived
  genotype each round;
* ``train`` — the genotype-built ``NetworkCIFAR`` (``models/cv/darts/eval_net.py``) trains its weights
  only; the server averages weights (FedNASAggregator.aggregate :66-74)."""
import logging

from ...trainers.nas import ModelTrainerNAS
from .fl_protocol import FedAVGAggregator, run_fl


class FedNASAggregator(FedAVGAggregator):
    def aggregate(self):
        averaged = super().aggregate()
        model = self.trainer.model
        if hasattr(model, "arch_parameters"):
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
        m = model_trainer.model
        out["genotype"] = m.genotype() if hasattr(m, "arch_parameters") else getattr(m, "genotype_used", None)
    return out
