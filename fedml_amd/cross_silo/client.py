"""``fedml_amd.cross_silo.Client`` (reference: `cross_silo/client.py:4-22`); the client rank
(``args.rank``) starts at 1."""
from .horizontal.fedml_server_manager import federation_size


class Client:
    def __init__(self, args, device, dataset, model, model_trainer=None, comm=None):
        if str(args.federated_optimizer) not in ("FedAvg", "FedAvgM", "FedOpt"):
            raise ValueError(f"cross-silo client supports FedAvg-style optimizers, got {args.federated_optimizer}")
        size = federation_size(args)
        scenario = str(getattr(args, "scenario", "horizontal"))
        rank = int(getattr(args, "rank", 1))
        if scenario == "hierarchical":
            from .hierarchical.fedml_hierarchical_api import init_client
            self.manager = init_client(args, device, comm, rank, size, model, dataset, model_trainer)
        else:
            from .horizontal import FedML_Horizontal
            self.manager = FedML_Horizontal(args, rank, size, comm, device, dataset, model, model_trainer)

    def run(self):
        self.manager.run()
