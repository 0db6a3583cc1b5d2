"""Silo master / slave roles (reference: `cross_silo/hierarchical/client_master_manager.py:48-269`,
`client_slave_manager.py:9-56`).

The master (process 0 of the silo) speaks the cross-silo protocol with the server. After every
``S2C_INIT_CONFIG`` / ``S2C_SYNC_MODEL_TO_CLIENT`` it broadcasts a 3-int header
``[round_idx, silo_index, finished]`` and then the flat model to the silo's other processes, and
all of them train one data-parallel round together. Slaves just loop on that header."""
import logging

import torch
import torch.distributed as dist

from ..horizontal.fedml_client_manager import FedMLClientManager
from ..message_define import MyMessage


def _bcast_header(round_idx, silo_index, finished, device):
    h = torch.tensor([round_idx, silo_index, finished], dtype=torch.int64, device=device)
    dist.broadcast(h, 0)
    return [int(v) for v in h.tolist()]


class ClientMasterManager(FedMLClientManager):
    """``trainer`` is a ``TrainerDistAdapter``."""

    def _pg_device(self):
        return self.trainer.device if self.trainer.device.type == "cuda" else torch.device("cpu")

    def _sync_silo(self, finished=False, silo=0):
        if self.trainer.n_proc > 1:
            _bcast_header(self.round_idx, silo, int(finished), self._pg_device())
            if not finished:
                self.trainer.sync_model()

    def handle_message_init(self, msg):
        params = self.resolve_payload(msg.get(MyMessage.MSG_ARG_KEY_MODEL_PARAMS))
        if self.plane_skip():       # RCCL plane, not selected this round: zeros into the reduce, no silo round
            return
        self.note_global(params)
        self.trainer.update_model(params)
        silo = int(msg.get(MyMessage.MSG_ARG_KEY_CLIENT_INDEX))
        self.round_idx = int(msg.get(MyMessage.MSG_ARG_KEY_ROUND_INDEX, 0))
        self._sync_silo(False, silo)
        self.trainer.update_dataset(silo)
        self._train_and_send()

    def handle_message_receive_model_from_server(self, msg):
        params = self.resolve_payload(msg.get(MyMessage.MSG_ARG_KEY_MODEL_PARAMS))
        if self.plane_skip():
            return
        self.note_global(params)
        self.trainer.update_model(params)
        silo = int(msg.get(MyMessage.MSG_ARG_KEY_CLIENT_INDEX))
        self.round_idx = int(msg.get(MyMessage.MSG_ARG_KEY_ROUND_INDEX, self.round_idx + 1))
        self._sync_silo(False, silo)
        self.trainer.update_dataset(silo)
        self._train_and_send()

    def handle_finish(self, msg):
        self._sync_silo(True)
        super().handle_finish(msg)
        self.trainer.cleanup_pg()

    def _train_and_send(self):
        # device plane: keep the silo average on the GPU (no state-dict round trip through the host)
        weights, n = self.trainer.train(self.round_idx, flat=self.mailbox is not None or self.plane is not None)
        self.send_model_to_server(0, weights, n)


class ClientSlaveManager:
    def __init__(self, args, trainer):
        self.args = args
        self.trainer = trainer
        self.rounds = 0

    def run(self):
        dev = self.trainer.device if self.trainer.device.type == "cuda" else torch.device("cpu")
        while True:
            round_idx, silo, finished = _bcast_header(0, 0, 0, dev)
            if finished:
                break
            self.trainer.sync_model()
            self.trainer.update_dataset(silo)
            self.trainer.train(round_idx)
            self.rounds += 1
        logging.info("silo slave %d finished after %d rounds", self.trainer.rank_in_silo, self.rounds)
        self.trainer.cleanup_pg()
