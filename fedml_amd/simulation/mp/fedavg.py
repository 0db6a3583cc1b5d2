"""FedAvg, message-passing (reference: `mpi_p2p_mp/fedavg/FedAvgAPI.py:19-168`)."""
from .fl_protocol import (FedAVGAggregator, FedAVGTrainer, FedAvgClientManager, FedAvgServerManager, MyMessage,
                          run_fl)


def FedML_FedAvg_distributed(args, process_id, worker_number, comm, device, dataset, model, model_trainer=None,
                             preprocessed_sampling_lists=None):
    return run_fl(args, process_id, worker_number, comm, device, dataset, model, model_trainer,
                  preprocessed_sampling_lists=preprocessed_sampling_lists)


__all__ = ["FedML_FedAvg_distributed", "FedAVGAggregator", "FedAVGTrainer", "FedAvgServerManager",
           "FedAvgClientManager", "MyMessage"]
