"""The server/client FedAvg protocol shared by the message-passing algorithms
(reference: `mpi_p2p_mp/fedavg/{FedAvgAPI,FedAvgServerManager,FedAvgClientManager,FedAVGAggregator,
FedAVGTrainer}.py` and their near-identical copies in fedopt/, fedprox/, fedavg_robust/).

Round structure: server samples clients (``np.random.seed(round)``) → S2C_INIT_CONFIG /
S2C_SYNC_MODEL_TO_CLIENT with the global model + client index to each worker → workers
train on that client's data → C2S_SEND_MODEL_TO_SERVER (params, num_samples) → once all
arrived the aggregator averages (flat arena + HIP kernel), optionally tests, and the next
round starts. Aggregation / optimisation behaviour is supplied by the aggregator and trainer
classes so FedAvg / FedOpt / FedProx / FedAvg-robust reuse one state machine.
"""
import logging
import time

import torch

from ...core.arena import ParamLayout, fedavg_state_dicts, stack_state_dicts
from ...core.distributed import ClientManager, Message, ServerManager
from ...core.mlops import MLOpsMetrics, MLOpsProfilerEvent
from ...trainers import create_model_trainer
from ..common import client_sampling, summarize_metrics


class MyMessage:
    MSG_TYPE_S2C_INIT_CONFIG = 1
    MSG_TYPE_S2C_SYNC_MODEL_TO_CLIENT = 2
    MSG_TYPE_C2S_SEND_MODEL_TO_SERVER = 3
    MSG_TYPE_C2S_SEND_STATS_TO_SERVER = 4
    MSG_TYPE_S2C_FINISH = 5

    MSG_ARG_KEY_TYPE = "msg_type"
    MSG_ARG_KEY_SENDER = "sender"
    MSG_ARG_KEY_RECEIVER = "receiver"
    MSG_ARG_KEY_NUM_SAMPLES = "num_samples"
    MSG_ARG_KEY_MODEL_PARAMS = "model_params"
    MSG_ARG_KEY_CLIENT_INDEX = "client_idx"
    MSG_ARG_KEY_ROUND_INDEX = "round_idx"
    MSG_ARG_KEY_TRAIN_CORRECT = "train_correct"
    MSG_ARG_KEY_TRAIN_ERROR = "train_error"
    MSG_ARG_KEY_TRAIN_NUM = "train_num_sample"
    MSG_ARG_KEY_TEST_CORRECT = "test_correct"
    MSG_ARG_KEY_TEST_ERROR = "test_error"
    MSG_ARG_KEY_TEST_NUM = "test_num_sample"


# ------------------------------------------------------------------------------------------------
class FedAVGAggregator:
    def __init__(self, train_global, test_global, all_train_data_num, train_data_local_dict, test_data_local_dict,
                 train_data_local_num_dict, worker_num, device, args, model_trainer):
        self.trainer = model_trainer
        self.args = args
        self.train_global = train_global
        self.test_global = test_global
        self.all_train_data_num = all_train_data_num
        self.train_data_local_dict = train_data_local_dict
        self.test_data_local_dict = test_data_local_dict
        self.train_data_local_num_dict = train_data_local_num_dict
        self.worker_num = worker_num
        self.device = device
        self.model_dict = {}
        self.sample_num_dict = {}
        self.flag_client_model_uploaded_dict = {i: False for i in range(worker_num)}
        self.history = []

    def get_global_model_params(self):
        return self.trainer.get_model_params()

    def set_global_model_params(self, model_parameters):
        self.trainer.set_model_params(model_parameters)

    def add_local_trained_result(self, index, model_params, sample_num):
        self.model_dict[index] = model_params
        self.sample_num_dict[index] = sample_num
        self.flag_client_model_uploaded_dict[index] = True

    def check_whether_all_receive(self):
        if not all(self.flag_client_model_uploaded_dict[i] for i in range(self.worker_num)):
            return False
        for i in range(self.worker_num):
            self.flag_client_model_uploaded_dict[i] = False
        return True

    def _w_locals(self):
        return [(self.sample_num_dict[i], self.model_dict[i]) for i in range(self.worker_num)]

    def aggregate(self):
        t0 = time.time()
        averaged = fedavg_state_dicts(self._w_locals())
        self.set_global_model_params(averaged)
        logging.info("aggregate time cost: %.3f s", time.time() - t0)
        return averaged

    def client_sampling(self, round_idx, client_num_in_total, client_num_per_round):
        return client_sampling(round_idx, client_num_in_total, client_num_per_round)

    def test_on_server_for_all_clients(self, round_idx):
        freq = int(getattr(self.args, "frequency_of_the_test", 0) or 0)
        last = round_idx == int(self.args.comm_round) - 1
        if not (last or (freq > 0 and round_idx % freq == 0)):
            return None
        tr, te = [], []
        for cid in range(int(self.args.client_num_in_total)):
            if cid in self.train_data_local_dict:
                tr.append(self.trainer.test(self.train_data_local_dict[cid], self.device, self.args))
            if cid in self.test_data_local_dict:
                te.append(self.trainer.test(self.test_data_local_dict[cid], self.device, self.args))
        tr_acc, tr_loss = summarize_metrics(tr)
        te_acc, te_loss = summarize_metrics(te)
        stats = {"round": round_idx, "Train/Acc": tr_acc, "Train/Loss": tr_loss, "Test/Acc": te_acc,
                 "Test/Loss": te_loss}
        self.history.append(stats)
        MLOpsMetrics.get_instance().log(stats, step=round_idx)
        logging.info("server test: %s", stats)
        return stats


class FedAVGTrainer:
    def __init__(self, client_index, train_data_local_dict, train_data_local_num_dict, test_data_local_dict,
                 train_data_num, device, args, model_trainer):
        self.trainer = model_trainer
        self.client_index = client_index
        self.train_data_local_dict = train_data_local_dict
        self.train_data_local_num_dict = train_data_local_num_dict
        self.test_data_local_dict = test_data_local_dict
        self.all_train_data_num = train_data_num
        self.train_local = None
        self.local_sample_number = None
        self.test_local = None
        self.device = device
        self.args = args

    def update_model(self, weights):
        self.trainer.set_model_params(weights)

    def update_dataset(self, client_index):
        self.client_index = client_index
        self.train_local = self.train_data_local_dict[client_index]
        self.local_sample_number = self.train_data_local_num_dict[client_index]
        self.test_local = self.test_data_local_dict.get(client_index)
        self.trainer.set_id(client_index)

    def train(self, round_idx=None):
        self.args.round_idx = round_idx
        self.trainer.train(self.train_local, self.device, self.args)
        return self.trainer.get_model_params(), self.local_sample_number


# ------------------------------------------------------------------------------------------------
class FedAvgServerManager(ServerManager):
    def __init__(self, args, aggregator, comm=None, rank=0, size=0, backend="LOOPBACK", is_preprocessed=False,
                 preprocessed_client_lists=None):
        super().__init__(args, comm, rank, size, backend)
        self.aggregator = aggregator
        self.round_num = int(args.comm_round)
        self.round_idx = 0
        self.is_preprocessed = is_preprocessed
        self.preprocessed_client_lists = preprocessed_client_lists
        self.round_times = []
        self._t0 = None

    def run(self):
        super().run()

    def _sample(self, round_idx):
        if self.is_preprocessed and self.preprocessed_client_lists is not None:
            return list(self.preprocessed_client_lists[round_idx])
        return self.aggregator.client_sampling(round_idx, int(self.args.client_num_in_total), self.size - 1)

    def send_init_msg(self):
        self._t0 = time.time()
        client_indexes = self._sample(self.round_idx)
        global_model_params = self.aggregator.get_global_model_params()
        for process_id in range(1, self.size):
            self.send_message_init_config(process_id, global_model_params, client_indexes[process_id - 1])

    def register_message_receive_handlers(self):
        self.register_message_receive_handler(MyMessage.MSG_TYPE_C2S_SEND_MODEL_TO_SERVER,
                                              self.handle_message_receive_model_from_client)

    def handle_message_receive_model_from_client(self, msg_params):
        sender_id = msg_params.get(MyMessage.MSG_ARG_KEY_SENDER)
        model_params = msg_params.get(MyMessage.MSG_ARG_KEY_MODEL_PARAMS)
        local_sample_number = msg_params.get(MyMessage.MSG_ARG_KEY_NUM_SAMPLES)
        self.aggregator.add_local_trained_result(sender_id - 1, model_params, local_sample_number)
        if not self.aggregator.check_whether_all_receive():
            return
        prof = MLOpsProfilerEvent.get_instance()
        prof.log_event_started("aggregate", event_value=str(self.round_idx))
        global_model_params = self.aggregator.aggregate()
        prof.log_event_ended("aggregate", event_value=str(self.round_idx))
        self.aggregator.test_on_server_for_all_clients(self.round_idx)
        now = time.time()
        self.round_times.append(now - self._t0)
        self._t0 = now
        self.round_idx += 1
        if self.round_idx == self.round_num:
            for pid in range(1, self.size):
                self.send_message(Message(MyMessage.MSG_TYPE_S2C_FINISH, self.get_sender_id(), pid))
            self.finish()
            return
        client_indexes = self._sample(self.round_idx)
        for receiver_id in range(1, self.size):
            self.send_message_sync_model_to_client(receiver_id, global_model_params, client_indexes[receiver_id - 1])

    def send_message_init_config(self, receive_id, global_model_params, client_index):
        m = Message(MyMessage.MSG_TYPE_S2C_INIT_CONFIG, self.get_sender_id(), receive_id)
        m.add_params(MyMessage.MSG_ARG_KEY_MODEL_PARAMS, global_model_params)
        m.add_params(MyMessage.MSG_ARG_KEY_CLIENT_INDEX, str(client_index))
        m.add_params(MyMessage.MSG_ARG_KEY_ROUND_INDEX, self.round_idx)
        self.send_message(m)

    def send_message_sync_model_to_client(self, receive_id, global_model_params, client_index):
        m = Message(MyMessage.MSG_TYPE_S2C_SYNC_MODEL_TO_CLIENT, self.get_sender_id(), receive_id)
        m.add_params(MyMessage.MSG_ARG_KEY_MODEL_PARAMS, global_model_params)
        m.add_params(MyMessage.MSG_ARG_KEY_CLIENT_INDEX, str(client_index))
        m.add_params(MyMessage.MSG_ARG_KEY_ROUND_INDEX, self.round_idx)
        self.send_message(m)


class FedAvgClientManager(ClientManager):
    def __init__(self, args, trainer, comm=None, rank=0, size=0, backend="LOOPBACK"):
        super().__init__(args, comm, rank, size, backend)
        self.trainer = trainer
        self.num_rounds = int(args.comm_round)
        self.round_idx = 0

    def register_message_receive_handlers(self):
        self.register_message_receive_handler(MyMessage.MSG_TYPE_S2C_INIT_CONFIG, self.handle_message_init)
        self.register_message_receive_handler(MyMessage.MSG_TYPE_S2C_SYNC_MODEL_TO_CLIENT,
                                              self.handle_message_receive_model_from_server)
        self.register_message_receive_handler(MyMessage.MSG_TYPE_S2C_FINISH, lambda m: self.finish())

    def handle_message_init(self, msg_params):
        self.trainer.update_model(msg_params.get(MyMessage.MSG_ARG_KEY_MODEL_PARAMS))
        self.trainer.update_dataset(int(msg_params.get(MyMessage.MSG_ARG_KEY_CLIENT_INDEX)))
        self.round_idx = int(msg_params.get(MyMessage.MSG_ARG_KEY_ROUND_INDEX, 0))
        self.__train()

    def handle_message_receive_model_from_server(self, msg_params):
        self.trainer.update_model(msg_params.get(MyMessage.MSG_ARG_KEY_MODEL_PARAMS))
        self.trainer.update_dataset(int(msg_params.get(MyMessage.MSG_ARG_KEY_CLIENT_INDEX)))
        self.round_idx = int(msg_params.get(MyMessage.MSG_ARG_KEY_ROUND_INDEX, self.round_idx + 1))
        self.__train()

    def send_model_to_server(self, receive_id, weights, local_sample_num):
        m = Message(MyMessage.MSG_TYPE_C2S_SEND_MODEL_TO_SERVER, self.get_sender_id(), receive_id)
        m.add_params(MyMessage.MSG_ARG_KEY_MODEL_PARAMS, weights)
        m.add_params(MyMessage.MSG_ARG_KEY_NUM_SAMPLES, local_sample_num)
        self.send_message(m)

    def __train(self):
        prof = MLOpsProfilerEvent.get_instance()
        prof.log_event_started("train", event_value=str(self.round_idx))
        weights, n = self.trainer.train(self.round_idx)
        prof.log_event_ended("train", event_value=str(self.round_idx))
        self.send_model_to_server(0, weights, n)


# ------------------------------------------------------------------------------------------------
def run_fl(args, process_id, worker_number, comm, device, dataset, model, model_trainer=None,
           aggregator_cls=FedAVGAggregator, trainer_cls=FedAVGTrainer, server_cls=FedAvgServerManager,
           client_cls=FedAvgClientManager, preprocessed_sampling_lists=None):
    (train_data_num, test_data_num, train_data_global, test_data_global, train_data_local_num_dict,
     train_data_local_dict, test_data_local_dict, class_num) = dataset[:8]
    backend = str(getattr(args, "backend", "LOOPBACK"))
    if backend.upper() == "MPI" and comm is not None:
        backend = "LOOPBACK"
    if model_trainer is None:
        model_trainer = create_model_trainer(model, args)
    model_trainer.set_id(process_id)
    if process_id == 0:
        aggregator = aggregator_cls(train_data_global, test_data_global, train_data_num, train_data_local_dict,
                                    test_data_local_dict, train_data_local_num_dict, worker_number - 1, device, args,
                                    model_trainer)
        server = server_cls(args, aggregator, comm, process_id, worker_number, backend,
                            is_preprocessed=preprocessed_sampling_lists is not None,
                            preprocessed_client_lists=preprocessed_sampling_lists)
        server.send_init_msg()
        server.run()
        return {"global_model": aggregator.get_global_model_params(), "history": aggregator.history,
                "round_times": server.round_times}
    trainer = trainer_cls(process_id - 1, train_data_local_dict, train_data_local_num_dict, test_data_local_dict,
                          train_data_num, device, args, model_trainer)
    client = client_cls(args, trainer, comm, process_id, worker_number, backend)
    client.run()
    return None
