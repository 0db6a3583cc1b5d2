"""Hierarchical cross-silo entry (reference: `cross_silo/hierarchical/fedml_hierarchical_api.py:18-255`):
rank 0 is the server (same protocol/aggregator as horizontal); silo ranks run a
``TrainerDistAdapter`` and, on the silo's process 0, the ``ClientMasterManager`` (others run
``ClientSlaveManager``)."""
from ...trainers import create_model_trainer
from ..horizontal.fedml_horizontal_api import _backend
from ..horizontal.fedml_horizontal_api import init_server as _init_server
from .client_manager import ClientMasterManager, ClientSlaveManager
from .trainer_dist_adapter import TrainerDistAdapter


def init_server(args, device, comm, rank, size, model, dataset, model_trainer=None, server_aggregator=None):
    return _init_server(args, device, comm, rank, size, model, dataset, model_trainer, server_aggregator)


def init_client(args, device, comm, rank, size, model, dataset, model_trainer=None):
    (train_num, _, _, _, num_dict, train_local, test_local, _) = dataset[:8]
    adapter = TrainerDistAdapter(args, device, rank, model, train_num, num_dict, train_local, test_local,
                                 model_trainer)
    if adapter.rank_in_silo == 0:
        return ClientMasterManager(args, adapter, comm, rank, size, _backend(args, comm))
    return ClientSlaveManager(args, adapter)


def FedML_Hierarchical(args, client_rank, client_num, comm, device, dataset, model, model_trainer=None,
                       server_aggregator=None):
    if client_rank == 0:
        return init_server(args, device, comm, 0, client_num, model, dataset, model_trainer, server_aggregator)
    return init_client(args, device, comm, client_rank, client_num, model, dataset, model_trainer)
