"""FedGAN over message passing (reference: `mpi_p2p_mp/fedgan/*`): the FedAvg state machine with
a GAN client trainer; generator and discriminator weights are averaged separately (they are
disjoint key sets of the ``MNISTGAN`` state dict)."""
from ...trainers.gan import ModelTrainerGAN
from .fl_protocol import run_fl


def FedML_FedGan_distributed(args, process_id, worker_number, comm, device, dataset, model, model_trainer=None,
                             preprocessed_sampling_lists=None):
    if model_trainer is None or not isinstance(model_trainer, ModelTrainerGAN):
        model_trainer = ModelTrainerGAN(model, args)
    return run_fl(args, process_id, worker_number, comm, device, dataset, model, model_trainer,
                  preprocessed_sampling_lists=preprocessed_sampling_lists)
