"""Cross-silo client state machine (reference: `cross_silo/horizontal/fedml_client_manager.py:14-173`).

On connection-ready: report ONLINE, start a system-metrics reporter (a daemon thread sampling
CPU / host memory / GPU utilisation via rocm-smi every ``sys_perf_interval`` seconds — the
reference forks a process). On init / sync: load the global model, switch to the assigned
data silo, train, upload (tensors travel as raw frames; no tensor→list conversion).
"""
import json
import logging
import platform
import threading
import time

import torch

from ...core.distributed import ClientManager, Message
from ...core.fault import FaultInjector
from ...core.mlops import MLOpsMetrics, MLOpsProfilerEvent
from ..message_define import MyMessage
from .fedml_server_manager import inject_connection_ready, parse_client_ids


class FedMLClientManager(ClientManager):
    def __init__(self, args, trainer, comm=None, client_rank=0, client_num=0, backend="TCP"):
        super().__init__(args, comm, client_rank, client_num, backend)
        self.trainer = trainer
        self.num_rounds = int(args.comm_round)
        self.round_idx = 0
        self.client_real_ids = parse_client_ids(args, client_num - 1)
        self.client_real_id = self.client_real_ids[self.get_sender_id() - 1]
        self.has_sent_online_msg = False
        self.mailbox = None
        self.plane = None            # RCCL data plane (cross_silo/fed_plane.py), opened by the first 'rccl' marker
        self._plane_train = True
        self._stop_stats = threading.Event()
        self.final_model = None
        self.faults = FaultInjector(args)
        # compressed uploads on the WAN path (cross_silo/wan_codec.py): int8 Δ + error feedback
        wc = str(getattr(args, "wan_compression", "") or "").lower()
        self.wan = None
        if wc:
            from ..wan_codec import WanEncoder
            dev = getattr(trainer, "device", None)   # the silo's GPU: quantisation runs as the HIP kernel
            self.wan = WanEncoder(wc, device=dev if dev is not None and torch.device(dev).type == "cuda" else None)

    def note_global(self, params):
        """The round's global model (the reference point of a compressed upload)."""
        if self.wan is not None and params is not None and not torch.is_tensor(params):
            self.wan.note_global(params)

    def resolve_payload(self, params):
        """A device-plane marker (``cross_silo/device_mailbox.py``) → the global model as a flat device
        tensor read from the server's shared buffer; any other payload passes through."""
        from ..device_mailbox import SiloMailbox, is_marker
        if not is_marker(params):
            return params
        if params["__devmail__"] == "rccl":
            return self._plane_receive(params)
        if self.mailbox is None or params["__devmail__"] == "init":
            if "desc" not in params:
                raise RuntimeError("device-plane marker without a mailbox descriptor before the silo opened one")
            self.mailbox = SiloMailbox(params["desc"], int(params["slot"]))
        return self.mailbox.glob

    def _plane_device(self):
        dev = getattr(self.trainer, "device", None)
        return torch.device(dev) if dev is not None and torch.device(dev).type == "cuda" else torch.device("cpu")

    def _plane_receive(self, mk):
        """Join the round's broadcast: the global model lands in this master's flat device buffer."""
        if self.plane is None:
            from ..fed_plane import FederationPlane
            rank = self.client_real_ids.index(self.client_real_id) + 1
            self.plane = FederationPlane(rank, len(self.client_real_ids) + 1, int(mk["port"]), self._plane_device())
            self._plane_buf = torch.zeros(int(mk["P"]), dtype=torch.float32, device=self._plane_device())
        self.plane.broadcast(self._plane_buf)
        self._plane_train = bool(mk.get("train", True))
        return self._plane_buf

    def finish(self):
        if self.plane is not None:      # release the RCCL plane's communicator and its store port
            self.plane.close()
            self.plane = None
        super().finish()

    def plane_skip(self):
        """RCCL plane, silo not selected this round: add zeros to the round's reduce and do nothing else."""
        if self.plane is None or self._plane_train:
            return False
        self.plane.reduce(torch.zeros(self._plane_buf.numel() + 1, dtype=torch.float32, device=self._plane_buf.device))
        return True

    def run(self):
        inject_connection_ready(self)
        super().run()

    def register_message_receive_handlers(self):
        self.register_message_receive_handler(MyMessage.MSG_TYPE_CONNECTION_IS_READY,
                                              self.handle_message_connection_ready)
        self.register_message_receive_handler(MyMessage.MSG_TYPE_S2C_INIT_CONFIG, self.handle_message_init)
        self.register_message_receive_handler(MyMessage.MSG_TYPE_S2C_SYNC_MODEL_TO_CLIENT,
                                              self.handle_message_receive_model_from_server)
        self.register_message_receive_handler(MyMessage.MSG_TYPE_S2C_FINISH, self.handle_finish)

    def handle_message_connection_ready(self, msg):
        if self.has_sent_online_msg:
            return
        self.has_sent_online_msg = True
        self.send_client_status(0)
        MLOpsMetrics.get_instance().report_client_training_status(self.client_real_id,
                                                                  MyMessage.MSG_MLOPS_CLIENT_STATUS_INITIALIZING)
        interval = float(getattr(self.args, "sys_perf_interval", 30.0) or 0)
        if interval > 0:
            threading.Thread(target=self.report_sys_performances, args=(interval,), daemon=True).start()

    def handle_message_init(self, msg):
        MLOpsMetrics.get_instance().report_client_training_status(self.client_real_id,
                                                                  MyMessage.MSG_MLOPS_CLIENT_STATUS_TRAINING)
        params = self.resolve_payload(msg.get(MyMessage.MSG_ARG_KEY_MODEL_PARAMS))
        self.round_idx = int(msg.get(MyMessage.MSG_ARG_KEY_ROUND_INDEX, 0))
        if self.plane_skip():
            return
        self.note_global(params)
        self.trainer.update_model(params)
        self.trainer.update_dataset(int(msg.get(MyMessage.MSG_ARG_KEY_CLIENT_INDEX)))
        self.__train()

    def handle_message_receive_model_from_server(self, msg):
        params = self.resolve_payload(msg.get(MyMessage.MSG_ARG_KEY_MODEL_PARAMS))
        self.round_idx = int(msg.get(MyMessage.MSG_ARG_KEY_ROUND_INDEX, self.round_idx + 1))
        if self.plane_skip():
            return
        self.note_global(params)
        self.trainer.update_model(params)
        self.trainer.update_dataset(int(msg.get(MyMessage.MSG_ARG_KEY_CLIENT_INDEX)))
        self.__train()

    def handle_finish(self, msg):
        params = self.resolve_payload(msg.get(MyMessage.MSG_ARG_KEY_MODEL_PARAMS))
        if params is not None:
            self.trainer.update_model(params)
            self.final_model = self.trainer.get_model_params() if torch.is_tensor(params) else params
        MLOpsMetrics.get_instance().report_client_training_status(self.client_real_id,
                                                                  MyMessage.MSG_MLOPS_CLIENT_STATUS_FINISHED)
        self._stop_stats.set()
        self.finish()

    def send_model_to_server(self, receive_id, weights, local_sample_num):
        MLOpsProfilerEvent.get_instance().log_event_started("comm_c2s", event_value=str(self.round_idx))
        m = Message(MyMessage.MSG_TYPE_C2S_SEND_MODEL_TO_SERVER, self.client_real_id, receive_id)
        plane_buf = None
        if self.plane is not None:
            # RCCL plane: n·w ‖ n goes into the round's reduce right after this marker (the server enters the
            # reduce once every selected silo's marker is in, so the marker must go first)
            from ..device_mailbox import marker
            if torch.is_tensor(weights):
                flat = weights
            elif hasattr(self.trainer, "flat_params"):
                flat = self.trainer.flat_params()
            else:
                from ...core.arena import ParamLayout
                flat = ParamLayout(weights).flatten(weights, device=self._plane_buf.device)
            n = float(local_sample_num)
            plane_buf = torch.empty(self._plane_buf.numel() + 1, dtype=torch.float32, device=self._plane_buf.device)
            torch.mul(flat.reshape(-1).to(plane_buf.device), n, out=plane_buf[:-1])
            plane_buf[-1:].fill_(n)
            weights = marker("rccl")
        elif getattr(self, "mailbox", None) is not None:
            # device plane: the upload goes into this silo's shared slot; the message only points at it
            from ..device_mailbox import marker
            if torch.is_tensor(weights):
                flat = weights
            elif hasattr(self.trainer, "flat_params"):
                flat = self.trainer.flat_params()
            else:
                from ...core.arena import ParamLayout
                flat = ParamLayout(weights).flatten(weights, device=self.mailbox.glob.device)
            self.mailbox.write_upload(flat, float(local_sample_num))
            weights = marker("slot", slot=self.mailbox.slot)
        elif self.wan is not None and self.wan.ref is not None:
            weights = self.wan.encode(weights, seed=self.round_idx * 4099 + int(self.client_real_id))
        m.add_params(MyMessage.MSG_ARG_KEY_MODEL_PARAMS, weights)
        m.add_params(MyMessage.MSG_ARG_KEY_NUM_SAMPLES, local_sample_num)
        m.add_params(MyMessage.MSG_ARG_KEY_ROUND_INDEX, self.round_idx)
        self.send_message(m)
        if plane_buf is not None:
            self.plane.reduce(plane_buf)

    def send_client_status(self, receive_id, status="ONLINE"):
        m = Message(MyMessage.MSG_TYPE_C2S_CLIENT_STATUS, self.client_real_id, receive_id)
        name = platform.system()
        m.add_params(MyMessage.MSG_ARG_KEY_CLIENT_STATUS, status)
        m.add_params(MyMessage.MSG_ARG_KEY_CLIENT_OS, "Mac" if name == "Darwin" else name)
        self.send_message(m)

    def report_sys_performances(self, interval):
        from ...core.mlops import SysStats
        stats = SysStats()
        while not self._stop_stats.wait(interval):
            try:
                MLOpsMetrics.get_instance().report_system_metric(stats.produce_info())
            except Exception:
                logging.debug("system metric sampling failed", exc_info=True)

    def __train(self):
        prof = MLOpsProfilerEvent.get_instance()
        prof.log_event_started("train", event_value=str(self.round_idx))
        weights, n = self.trainer.train(self.round_idx)
        prof.log_event_ended("train", event_value=str(self.round_idx))
        # injected faults (core.fault): a dropped client never uploads, a delayed one uploads late
        if self.faults.dropped(self.round_idx, self.client_real_id):
            logging.info("client %d: injected dropout in round %d", self.client_real_id, self.round_idx)
            return
        d = self.faults.delay(self.round_idx, self.client_real_id)
        if d > 0:
            time.sleep(d)
        self.send_model_to_server(0, weights, n)
