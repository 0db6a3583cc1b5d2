"""``fedml_amd.cross_silo.Server`` (reference: `cross_silo/server.py:4-23`)."""
from .horizontal.fedml_server_manager import federation_size


class Server:
    def __init__(self, args, device, dataset, model, model_trainer=None, server_aggregator=None, comm=None):
        if str(args.federated_optimizer) not in ("FedAvg", "FedAvgM", "FedOpt"):
            raise ValueError(f"cross-silo server supports FedAvg-style optimizers, got {args.federated_optimizer}")
        scenario = str(getattr(args, "scenario", "horizontal"))
        size = federation_size(args)
        if scenario == "hierarchical":
            from .hierarchical.fedml_hierarchical_api import init_server
            self.manager = init_server(args, device, comm, 0, size, model, dataset, model_trainer, server_aggregator)
        else:
            from .horizontal import FedML_Horizontal
            self.manager = FedML_Horizontal(args, 0, size, comm, device, dataset, model, model_trainer,
                                            server_aggregator)

    @property
    def aggregator(self):
        return self.manager.aggregator

    def run(self):
        self.manager.run()
        return self.manager.aggregator.get_global_model_params()
