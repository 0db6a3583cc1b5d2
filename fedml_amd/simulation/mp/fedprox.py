"""FedProx, message-passing (reference: `mpi_p2p_mp/fedprox/*` — there identical to FedAvg; here with the
real proximal term, ``fedprox_mu``/``mu``)."""
from ...trainers.fedprox import ModelTrainerFedProx
from .fl_protocol import run_fl


def FedML_FedProx_distributed(args, process_id, worker_number, comm, device, dataset, model, model_trainer=None,
                              preprocessed_sampling_lists=None):
    if model_trainer is None:
        model_trainer = ModelTrainerFedProx(model, args)
    return run_fl(args, process_id, worker_number, comm, device, dataset, model, model_trainer,
                  preprocessed_sampling_lists=preprocessed_sampling_lists)
