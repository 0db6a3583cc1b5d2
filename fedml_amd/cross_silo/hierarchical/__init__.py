from .client_manager import ClientMasterManager, ClientSlaveManager
from .fedml_hierarchical_api import FedML_Hierarchical, init_client, init_server
from .process_group_manager import ProcessGroupManager
from .trainer_dist_adapter import TrainerDistAdapter
from ..horizontal.fedml_server_manager import federation_size


class Server:
    def __init__(self, args, device, dataset, model, model_trainer=None, server_aggregator=None, comm=None):
        size = federation_size(args)
        self.manager = init_server(args, device, comm, 0, size, model, dataset, model_trainer, server_aggregator)

    def run(self):
        self.manager.run()
        return self.manager.aggregator.get_global_model_params()


class Client:
    def __init__(self, args, device, dataset, model, model_trainer=None, comm=None):
        size = federation_size(args)
        self.manager = init_client(args, device, comm, int(getattr(args, "rank", 1)), size, model, dataset,
                                   model_trainer)

    def run(self):
        self.manager.run()
