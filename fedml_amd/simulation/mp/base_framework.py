"""Minimal server/client skeleton (reference: `mpi_p2p_mp/base_framework/*`): each round the
clients send a local scalar result, the central worker aggregates (sum) and broadcasts it back."""
import random

from ...core.distributed import ClientManager, Message, ServerManager

MSG_C2S_RESULT = 1
MSG_S2C_GLOBAL = 2
MSG_S2C_FINISH = 3


class BaseCentralManager(ServerManager):
    def __init__(self, args, comm, rank, size, backend):
        super().__init__(args, comm, rank, size, backend)
        self.round = 0
        self.results = {}
        self.history = []

    def register_message_receive_handlers(self):
        self.register_message_receive_handler(MSG_C2S_RESULT, self.handle_result)

    def handle_result(self, msg):
        self.results[msg.get_sender_id()] = float(msg.get("result"))
        if len(self.results) < self.size - 1:
            return
        total = sum(self.results.values())
        self.history.append(total)
        self.results.clear()
        self.round += 1
        done = self.round >= int(self.args.comm_round)
        for r in range(1, self.size):
            m = Message(MSG_S2C_FINISH if done else MSG_S2C_GLOBAL, 0, r)
            m.add_params("global_result", total)
            self.send_message(m)
        if done:
            self.finish()


class BaseClientManager(ClientManager):
    def __init__(self, args, comm, rank, size, backend):
        super().__init__(args, comm, rank, size, backend)
        self.rng = random.Random(rank)

    def register_message_receive_handlers(self):
        self.register_message_receive_handler(MSG_S2C_GLOBAL, lambda m: self.send_result())
        self.register_message_receive_handler(MSG_S2C_FINISH, lambda m: self.finish())

    def send_result(self):
        m = Message(MSG_C2S_RESULT, self.rank, 0)
        m.add_params("result", self.rng.random())
        self.send_message(m)


def FedML_Base_distributed(args, process_id, worker_number, comm, device=None, dataset=None, model=None,
                           model_trainer=None, **_):
    backend = "LOOPBACK" if comm is not None else str(getattr(args, "backend", "TCP"))
    if process_id == 0:
        s = BaseCentralManager(args, comm, 0, worker_number, backend)
        s.run()
        return {"history": s.history}
    c = BaseClientManager(args, comm, process_id, worker_number, backend)
    c.send_result()
    c.run()
