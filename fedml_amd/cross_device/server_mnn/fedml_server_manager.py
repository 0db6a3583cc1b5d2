"""Cross-device (BeeHive) server manager (reference: `cross_device/server_mnn/fedml_server_manager.py:15-342`).

Publishes the ``start_train`` run description on ``flserver_agent/<edge_id>/start_train`` for every
device, waits for all devices to report ONLINE, then runs FedAvg rounds whose payload is a model
FILE path (MQTT_S3_MNN transport moves the bytes through the blob store)."""
import json
import logging
import time

from ...core.distributed import Message
from ...cross_silo.horizontal.fedml_server_manager import FedMLServerManager as _SiloServer
from ...cross_silo.horizontal.fedml_server_manager import parse_client_ids
from ..server_mnn.message_define import MyMessage


class FedMLServerManager(_SiloServer):
    def __init__(self, args, aggregator, comm=None, rank=0, size=0, backend="MQTT_S3_MNN", broker=None):
        super().__init__(args, aggregator, comm, rank, size, backend)
        self.broker = broker

    def start_train_payload(self):
        a = self.args
        return {
            "edges": [{"id": cid, "os_type": getattr(a, "client_os", "Android")} for cid in self.client_real_ids],
            "edgeids": self.client_real_ids, "runId": getattr(a, "run_id", "0"), "starttime": int(time.time() * 1000),
            "run_config": {"parameters": {
                "model_args": {"model": a.model, "global_model_file_path": self.aggregator.global_model_file_path,
                               "model_file_format": getattr(a, "model_file_format", "safetensors")},
                "train_args": {k: getattr(a, k, None) for k in (
                    "batch_size", "weight_decay", "client_num_per_round", "client_num_in_total", "comm_round",
                    "client_optimizer", "epochs", "learning_rate", "federated_optimizer")},
                "data_args": {k: getattr(a, k, None) for k in ("dataset", "partition_method", "partition_alpha")},
                "comm_args": {"backend": "MQTT_S3_MNN"}}},
        }

    def start_train(self):
        if self.broker is None:
            from ...core.distributed.communication.pubsub import default_broker
            self.broker = default_broker(self.args)
        payload = json.dumps(self.start_train_payload()).encode()
        for cid in self.client_real_ids:
            self.broker.publish(f"flserver_agent/{cid}/start_train", payload)
        logging.info("start_train published to %d devices", len(self.client_real_ids))

    def run(self):
        self.start_train()
        super().run()
