"""Cross-device server entry (reference: `cross_device/server_mnn/server_mnn_api.py:10-93`)."""
from ...cross_silo.horizontal.fedml_server_manager import federation_size
from ...trainers import create_model_trainer
from .fedml_aggregator import FedMLAggregator
from .fedml_server_manager import FedMLServerManager


def fedavg_cross_device(args, process_id, worker_number, comm, device, test_dataloader, model, model_trainer=None,
                        broker=None, train_data_num=0, train_data_local_num_dict=None):
    model_trainer = model_trainer or create_model_trainer(model, args)
    model_trainer.set_id(0)
    aggregator = FedMLAggregator(test_dataloader, train_data_num, train_data_local_num_dict or {}, worker_number - 1,
                                 device, args, model_trainer)
    backend = "LOOPBACK" if comm is not None and type(comm).__name__ == "LoopbackRouter" else \
        str(getattr(args, "backend", "MQTT_S3_MNN"))
    return FedMLServerManager(args, aggregator, comm, process_id, worker_number, backend, broker=broker)


class ServerMNN:
    def __init__(self, args, device, test_dataloader, model, model_trainer=None, comm=None, broker=None):
        if str(args.federated_optimizer) != "FedAvg":
            raise ValueError(f"cross-device server supports FedAvg, got {args.federated_optimizer}")
        if isinstance(test_dataloader, (list, tuple)) and len(test_dataloader) >= 8:
            test_dataloader = test_dataloader[3]  # the 8-tuple's global test set
        self.manager = fedavg_cross_device(args, 0, federation_size(args), comm, device, test_dataloader, model,
                                           model_trainer, broker)

    def run(self):
        self.manager.run()
        return self.manager.aggregator.get_global_model_params()
