"""Cross-silo server state machine (reference: `cross_silo/horizontal/fedml_server_manager.py:15-263`).

Handshake: every client reports ``C2S_CLIENT_STATUS = ONLINE``; when all ids of
``client_id_list`` are online the server sends ``S2C_INIT_CONFIG`` (global model + data-silo
index) to the round's selected clients. Each round: collect ``C2S_SEND_MODEL_TO_SERVER`` from
the selected clients, aggregate (flat-arena kernel), test, report round info, send
``S2C_SYNC_MODEL_TO_CLIENT``. After ``comm_round`` rounds the server stops (clients stop after
the final sync, as in the reference, and additionally on ``S2C_FINISH``).

Same-node device data plane (``silo_transport: device``; ``cross_silo/device_mailbox.py``): the model
payloads stay in HBM — the server publishes the global model into a HIP-IPC-shared buffer and aggregates
the silos' uploads straight from shared slots; the messages carry markers only.

Deadline rounds (not in the reference, which waits for every client forever): with
``round_timeout`` (seconds) the server closes a round when the deadline passes and aggregates the
uploads that arrived (at least ``min_clients_per_round``, default 1), re-weighted by their sample
counts; uploads tagged with an older round index are discarded.
"""
import json
import logging
import threading
import time

import torch

from ...core.distributed import Message, ServerManager
from ...core.mlops import MLOpsMetrics, MLOpsProfilerEvent
from ..message_define import MyMessage


def parse_client_ids(args, n_clients):
    ids = getattr(args, "client_id_list", None)
    if isinstance(ids, str) and ids.strip():
        return [int(v) for v in json.loads(ids)]
    if isinstance(ids, (list, tuple)) and ids:
        return [int(v) for v in ids]
    return list(range(1, n_clients + 1))


def federation_size(args):
    """Transport world = server + silos: from ``client_id_list`` when given, else
    ``client_num_per_round + 1`` (``worker_num`` in hierarchical mode counts silos only)."""
    ids = getattr(args, "client_id_list", None)
    if ids:
        return len(parse_client_ids(args, 0)) + 1
    return int(getattr(args, "client_num_per_round", 1)) + 1


class FedMLServerManager(ServerManager):
    def __init__(self, args, aggregator, comm=None, client_rank=0, client_num=0, backend="TCP",
                 is_preprocessed=False, preprocessed_client_lists=None):
        super().__init__(args, comm, client_rank, client_num, backend)
        self.aggregator = aggregator
        self.round_num = int(args.comm_round)
        self.round_idx = 0
        self.is_preprocessed = is_preprocessed
        self.preprocessed_client_lists = preprocessed_client_lists
        self.client_real_ids = parse_client_ids(args, client_num - 1)
        self.client_online_mapping = {}
        self.start_running_time = 0.0
        self.round_times = []
        self.test_times = []
        self._selected = []
        self._started = False
        to = getattr(args, "round_timeout", None)
        self.round_timeout = float(to) if to not in (None, "", 0, 0.0) else None
        self.min_clients = max(1, int(getattr(args, "min_clients_per_round", 1) or 1))
        self._timer = None
        self.partial_rounds = []     # (round, #arrived, #selected) of rounds closed by the deadline
        self.device_payload = str(getattr(args, "silo_transport", "") or "").lower() == "device"
        if self.device_payload and not torch.cuda.is_available():
            raise ValueError("silo_transport: device needs the GPU (HIP IPC buffers)")
        self.mailbox = None
        self._slot_of = {cid: i for i, cid in enumerate(self.client_real_ids)}
        # same-node RCCL data plane (cross_silo/fed_plane.py): one broadcast + one reduce per round
        self.rccl_payload = str(getattr(args, "silo_transport", "") or "").lower() == "rccl"
        if self.rccl_payload and self.round_timeout is not None:
            raise ValueError("silo_transport: rccl does not support round_timeout (a missing silo stalls the collective)")
        self.plane = None
        self._plane_glob = None

    def run(self):
        inject_connection_ready(self)
        super().run()

    # ------------------------------------------------------------------------------------------
    def register_message_receive_handlers(self):
        self.register_message_receive_handler(MyMessage.MSG_TYPE_CONNECTION_IS_READY, self.handle_connection_ready)
        self.register_message_receive_handler(MyMessage.MSG_TYPE_C2S_CLIENT_STATUS,
                                              self.handle_message_client_status_update)
        self.register_message_receive_handler(MyMessage.MSG_TYPE_C2S_SEND_MODEL_TO_SERVER,
                                              self.handle_message_receive_model_from_client)
        self.register_message_receive_handler(MyMessage.MSG_TYPE_ROUND_DEADLINE, self.handle_round_deadline)

    # ---- deadline rounds ---------------------------------------------------------------------------
    def _arm_deadline(self):
        if self.round_timeout is None:
            return
        if self._timer is not None:
            self._timer.cancel()
        r = self.round_idx

        def fire():   # delivered through the receive loop: handlers never run concurrently
            m = Message(MyMessage.MSG_TYPE_ROUND_DEADLINE, self.rank, self.rank)
            m.add_params(MyMessage.MSG_ARG_KEY_ROUND_INDEX, r)
            self.com_manager.deliver(m)
        self._timer = threading.Timer(self.round_timeout, fire)
        self._timer.daemon = True
        self._timer.start()

    def handle_round_deadline(self, msg):
        if int(msg.get(MyMessage.MSG_ARG_KEY_ROUND_INDEX)) != self.round_idx:
            return
        arrived = sum(1 for v in self.aggregator.flag_client_model_uploaded_dict.values() if v)
        if arrived < self.min_clients:
            logging.warning("round %d deadline: %d/%d uploads (< %d); extending", self.round_idx, arrived,
                            len(self._selected), self.min_clients)
            self._arm_deadline()
            return
        logging.warning("round %d deadline: aggregating %d of %d uploads", self.round_idx, arrived,
                        len(self._selected))
        self.partial_rounds.append((self.round_idx, arrived, len(self._selected)))
        for i in self.aggregator.flag_client_model_uploaded_dict:
            self.aggregator.flag_client_model_uploaded_dict[i] = False
        self._complete_round()

    def handle_connection_ready(self, msg):
        MLOpsMetrics.get_instance().report_server_training_status(getattr(self.args, "run_id", "0"),
                                                                  MyMessage.MSG_MLOPS_SERVER_STATUS_STARTING)

    def handle_message_client_status_update(self, msg):
        if msg.get(MyMessage.MSG_ARG_KEY_CLIENT_STATUS) == "ONLINE":
            self.client_online_mapping[int(msg.get_sender_id())] = True
        if not self._started and all(self.client_online_mapping.get(c, False) for c in self.client_real_ids):
            self._started = True
            MLOpsMetrics.get_instance().report_server_training_status(getattr(self.args, "run_id", "0"),
                                                                      MyMessage.MSG_MLOPS_SERVER_STATUS_RUNNING)
            self.send_init_msg()

    def _selection(self):
        ids = self.aggregator.client_selection(self.round_idx, self.client_real_ids,
                                               int(getattr(self.args, "client_num_per_round", len(self.client_real_ids))))
        silos = self.aggregator.data_silo_selection(self.round_idx, int(self.args.client_num_in_total), len(ids))
        return ids, silos

    def _open_mailbox(self, g):
        from ...core.arena import ParamLayout
        from ..device_mailbox import ServerMailbox
        layout = ParamLayout(g)
        self.mailbox = ServerMailbox(layout.size, len(self.client_real_ids), torch.device("cuda"))
        self.mailbox.publish(layout.flatten(g, device=self.mailbox.glob.device))
        self.aggregator.flat_layout = layout

    def send_init_msg(self):
        self.start_running_time = time.time()
        self._t0 = time.time()
        g = self.aggregator.get_global_model_params()
        ids, silos = self._selection()
        self._selected = ids
        self.aggregator.flag_client_model_uploaded_dict = {i: False for i in range(len(ids))}
        if self.rccl_payload:
            self._plane_round(MyMessage.MSG_TYPE_S2C_INIT_CONFIG, g, ids, silos)
            MLOpsProfilerEvent.get_instance().log_event_started("server.wait", event_value=str(self.round_idx))
            return
        if self.device_payload:
            from ..device_mailbox import marker
            self._open_mailbox(g)
            desc = self._desc = self.mailbox.descriptor()
        for cid, silo in zip(ids, silos):
            payload = marker("init", desc=desc, slot=self._slot_of[cid]) if self.device_payload else g
            self._send(MyMessage.MSG_TYPE_S2C_INIT_CONFIG, cid, payload, silo)
        MLOpsProfilerEvent.get_instance().log_event_started("server.wait", event_value=str(self.round_idx))
        self._arm_deadline()

    def finish(self):
        if self.plane is not None:      # release the RCCL plane's communicator and its store port
            self.plane.close()
            self.plane = None
        super().finish()

    # ---- RCCL data plane ------------------------------------------------------------------------
    def _plane_round(self, mtype, g, ids, silos, final=False):
        """Markers to EVERY silo (selected ones train on their data silo, the others only join the collectives),
        then the global model as one broadcast. ``g``: state dict or flat device tensor."""
        from ..device_mailbox import marker
        from ..fed_plane import FederationPlane, plane_port
        use_gpu = torch.cuda.is_available() and bool(getattr(self.args, "using_gpu", True))
        dev = torch.device("cuda") if use_gpu else torch.device("cpu")   # same device kind as the silo masters
        if self._plane_glob is None:
            from ...core.arena import ParamLayout
            layout = ParamLayout(g)
            self.aggregator.flat_layout = layout
            self._plane_glob = torch.zeros(layout.size, dtype=torch.float32, device=dev)
        if torch.is_tensor(g):
            self._plane_glob.copy_(g.reshape(-1))
        else:
            self.aggregator.flat_layout.flatten(g, out=self._plane_glob)
        P = self._plane_glob.numel()
        if getattr(self, "_plane_port", None) is None:
            self._plane_port = plane_port(self.args)
        port = self._plane_port
        silo_of = dict(zip(ids, silos))
        for cid in self.client_real_ids:
            mk = marker("rccl", P=P, port=port, train=cid in silo_of and not final)
            self._send(mtype if cid in silo_of or final else MyMessage.MSG_TYPE_S2C_SYNC_MODEL_TO_CLIENT, cid, mk,
                       silo_of.get(cid, 0))
        if self.plane is None:
            self.plane = FederationPlane(0, len(self.client_real_ids) + 1, port, dev)
        self.plane.broadcast(self._plane_glob)

    def _plane_aggregate(self):
        """Σ n·w ‖ Σ n of the round's selected silos (the others add zeros) by one reduce; w = the new global."""
        acc = torch.zeros(self._plane_glob.numel() + 1, dtype=torch.float32, device=self._plane_glob.device)
        self.plane.reduce(acc)
        avg = acc[:-1] / acc[-1:].clamp_min(1e-30)
        self.aggregator.model_dict.clear()
        self.aggregator.sample_num_dict.clear()
        self.aggregator._flat_global = avg
        return avg

    def _global_payload(self, g, cid):
        """Device plane: a 'global' marker that also carries the mailbox descriptor and the receiver's slot, so a
        silo left out of round 0 (partial participation: it never got the 'init' marker) can still open the
        shared buffers when it is first selected, or at FINISH."""
        if not self.device_payload:
            return g
        from ..device_mailbox import marker
        return marker("global", desc=self._desc, slot=self._slot_of[cid])

    def _send(self, mtype, receiver, params, silo):
        m = Message(mtype, self.get_sender_id(), receiver)
        m.add_params(MyMessage.MSG_ARG_KEY_MODEL_PARAMS, params)
        m.add_params(MyMessage.MSG_ARG_KEY_CLIENT_INDEX, str(silo))
        m.add_params(MyMessage.MSG_ARG_KEY_ROUND_INDEX, self.round_idx)
        self.send_message(m)

    def handle_message_receive_model_from_client(self, msg):
        sender = int(msg.get(MyMessage.MSG_ARG_KEY_SENDER))
        r = msg.get(MyMessage.MSG_ARG_KEY_ROUND_INDEX)
        if (r is not None and int(r) != self.round_idx) or sender not in self._selected:
            logging.info("discarding stale upload of client %d (round %s, server at %d)", sender, r, self.round_idx)
            return
        prof = MLOpsProfilerEvent.get_instance()
        prof.log_event_ended("comm_c2s", event_value=str(self.round_idx), event_edge_id=sender)
        params = msg.get(MyMessage.MSG_ARG_KEY_MODEL_PARAMS)
        from ..device_mailbox import is_marker
        from ..wan_codec import decode, is_encoded, payload_bytes
        if is_marker(params) and params.get("__devmail__") == "rccl":
            params = None        # RCCL plane: the upload arrives in the round's reduce, the marker only counts it
        elif is_marker(params):    # same-node device plane: the upload sits in the sender's shared slot
            params, _ = self.mailbox.upload(int(params["slot"]))
        else:
            self.wan_bytes = getattr(self, "wan_bytes", 0) + payload_bytes(params)
        if is_encoded(params):   # compressed silo update: w_global + deq(Δ) (cross_silo/wan_codec.py)
            params = decode(params, self.aggregator.get_global_model_params(),
                            device="cuda" if torch.cuda.is_available() else None)
        self.aggregator.add_local_trained_result(self._selected.index(sender), params,
                                                 msg.get(MyMessage.MSG_ARG_KEY_NUM_SAMPLES))
        if not self.aggregator.check_whether_all_receive():
            return
        self._complete_round()

    def _complete_round(self):
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None
        prof = MLOpsProfilerEvent.get_instance()
        prof.log_event_ended("server.wait", event_value=str(self.round_idx))
        prof.log_event_started("aggregate", event_value=str(self.round_idx))
        g = self._plane_aggregate() if self.rccl_payload else self.aggregator.aggregate()
        prof.log_event_ended("aggregate", event_value=str(self.round_idx))
        if torch.is_tensor(g) and g.is_cuda:
            torch.cuda.synchronize(g.device)
        now = time.time()   # the round's training + aggregation; server-side evaluation is timed on its own
        try:
            t_test = time.time()
            self.aggregator.test_on_server_for_all_clients(self.round_idx)
            self.test_times.append(time.time() - t_test)
        except Exception:  # evaluation must never stall the federation (reference behaviour)
            logging.exception("server-side test failed")
        self.round_times.append(now - self._t0)
        logging.info("round %d complete in %.3f s", self.round_idx, now - self._t0)
        self._t0 = time.time()
        MLOpsMetrics.get_instance().report_server_training_round_info(
            {"run_id": getattr(self.args, "run_id", "0"), "round_index": self.round_idx,
             "total_rounds": self.round_num, "running_time": round(now - self.start_running_time, 4)})
        self.round_idx += 1
        if self.device_payload:
            self.mailbox.publish(g if torch.is_tensor(g) else self.aggregator.flat_layout.flatten(
                g, device=self.mailbox.glob.device))
            g = None
        if self.rccl_payload:
            final = self.round_idx == self.round_num
            ids, silos = ([], []) if final else self._selection()
            self._selected = ids
            self.aggregator.flag_client_model_uploaded_dict = {i: False for i in range(len(ids))}
            self._plane_round(MyMessage.MSG_TYPE_S2C_FINISH if final else MyMessage.MSG_TYPE_S2C_SYNC_MODEL_TO_CLIENT,
                              g, ids, silos, final=final)
            if final:
                MLOpsMetrics.get_instance().report_server_training_status(
                    getattr(self.args, "run_id", "0"), MyMessage.MSG_MLOPS_SERVER_STATUS_FINISHED)
                self.finish()
            else:
                prof.log_event_started("server.wait", event_value=str(self.round_idx))
            return
        if self.round_idx == self.round_num:
            # final sync lets clients see the final model; then everyone stops
            for cid in self.client_real_ids:
                self._send(MyMessage.MSG_TYPE_S2C_FINISH, cid, self._global_payload(g, cid), 0)
            MLOpsMetrics.get_instance().report_server_training_status(getattr(self.args, "run_id", "0"),
                                                                      MyMessage.MSG_MLOPS_SERVER_STATUS_FINISHED)
            self.finish()
            return
        ids, silos = self._selection()
        self._selected = ids
        self.aggregator.flag_client_model_uploaded_dict = {i: False for i in range(len(ids))}
        for cid, silo in zip(ids, silos):
            self._send(MyMessage.MSG_TYPE_S2C_SYNC_MODEL_TO_CLIENT, cid, self._global_payload(g, cid), silo)
        prof.log_event_started("server.wait", event_value=str(self.round_idx))
        self._arm_deadline()


def inject_connection_ready(mgr):
    """Transports without a broker (loopback, TCP, gRPC) get the local CONNECTION_IS_READY the
    MQTT transport emits on connect (`mqtt_s3_multi_clients_comm_manager.py:175-180`)."""
    from ...core.distributed.communication.pubsub import MqttS3CommManager
    if not isinstance(mgr.com_manager, MqttS3CommManager):
        mgr.com_manager.deliver(Message(MyMessage.MSG_TYPE_CONNECTION_IS_READY, mgr.rank, mgr.rank))
