"""SplitNN over message passing (reference: `mpi_p2p_mp/split_nn/*`, Vepakomma et al. 2018).

Each client owns the bottom of the network, the server owns the top. A semaphore circulates
through clients ``1 → 2 → … → N → 1``; the holder runs one local epoch: forward its bottom
half, ship ``(activations, labels)`` (C2S_SEND_ACTS), the server does forward + backward of
the top half and returns ``∂L/∂activations`` (S2C_GRADS), the client back-propagates that
into its bottom half. Then a validation pass (C2S_VALIDATION_MODE … C2S_VALIDATION_OVER),
then the semaphore moves on. After ``epochs`` turns the last client sends
C2S_PROTOCOL_FINISHED and the server stops everyone.

``model`` is the pair ``(client_model, server_model)``. Optimiser: SGD(lr, momentum 0.9,
wd 5e-4) on both halves like the reference.
"""
import logging

import torch
import torch.nn as nn

from ...core.distributed import ClientManager, Message, ServerManager

MSG_S2C_GRADS = 1
MSG_C2S_SEND_ACTS = 2
MSG_C2S_VALIDATION_MODE = 3
MSG_C2S_VALIDATION_OVER = 4
MSG_C2S_PROTOCOL_FINISHED = 5
MSG_C2C_SEMAPHORE = 6
MSG_S2C_FINISH = 7


def _sgd(params, args):
    return torch.optim.SGD(params, lr=float(getattr(args, "learning_rate", 0.1)), momentum=0.9, weight_decay=5e-4)


class SplitNNServer:
    def __init__(self, model, max_rank, device, args):
        self.model = model.to(device)
        self.device = device
        self.args = args
        self.max_rank = max_rank
        self.optimizer = _sgd(self.model.parameters(), args)
        self.criterion = nn.CrossEntropyLoss()
        self.phase = "train"
        self.reset_stats()
        self.history = []

    def reset_stats(self):
        self.total = self.correct = 0
        self.loss_sum = 0.0
        self.steps = 0

    def forward_backward(self, acts, labels):
        acts = acts.to(self.device).float().requires_grad_(self.phase == "train")
        labels = labels.to(self.device)
        if self.phase == "train":
            self.model.train()
            self.optimizer.zero_grad(set_to_none=True)
            out = self.model(acts)
            loss = self.criterion(out, labels)
            loss.backward()
            self.optimizer.step()
            grads = acts.grad.detach().cpu()
        else:
            self.model.eval()
            with torch.no_grad():
                out = self.model(acts)
                loss = self.criterion(out, labels)
            grads = None
        self.total += labels.numel()
        self.correct += int((out.argmax(1) == labels).sum())
        self.loss_sum += float(loss.detach())
        self.steps += 1
        return grads

    def validation_over(self, client):
        stats = {"client": client, "val_acc": self.correct / max(1, self.total),
                 "val_loss": self.loss_sum / max(1, self.steps)}
        self.history.append(stats)
        logging.info("SplitNN validation: %s", stats)
        self.phase = "train"
        self.reset_stats()


class SplitNNServerManager(ServerManager):
    def __init__(self, args, server, comm, rank, size, backend):
        super().__init__(args, comm, rank, size, backend)
        self.server = server

    def register_message_receive_handlers(self):
        self.register_message_receive_handler(MSG_C2S_SEND_ACTS, self.handle_acts)
        self.register_message_receive_handler(MSG_C2S_VALIDATION_MODE, self.handle_val_mode)
        self.register_message_receive_handler(MSG_C2S_VALIDATION_OVER, self.handle_val_over)
        self.register_message_receive_handler(MSG_C2S_PROTOCOL_FINISHED, self.handle_finished)

    def handle_acts(self, msg):
        grads = self.server.forward_backward(msg.get("activations"), msg.get("labels"))
        if grads is not None:
            m = Message(MSG_S2C_GRADS, 0, msg.get_sender_id())
            m.add_params("grads", grads)
            self.send_message(m)

    def handle_val_mode(self, msg):
        self.server.reset_stats()
        self.server.phase = "validation"

    def handle_val_over(self, msg):
        self.server.validation_over(msg.get_sender_id())

    def handle_finished(self, msg):
        for r in range(1, self.size):
            self.send_message(Message(MSG_S2C_FINISH, 0, r))
        self.finish()


class SplitNNClient:
    def __init__(self, model, train_data, test_data, device, args):
        self.model = model.to(device)
        self.train_data = train_data
        self.test_data = test_data
        self.device = device
        self.optimizer = _sgd(self.model.parameters(), args)
        self.acts = None


class SplitNNClientManager(ClientManager):
    def __init__(self, args, client, comm, rank, size, backend):
        super().__init__(args, comm, rank, size, backend)
        self.client = client
        self.max_rank = size - 1
        self.epochs = int(getattr(args, "epochs", 1))
        self.turns_done = 0
        self._it = None

    def register_message_receive_handlers(self):
        self.register_message_receive_handler(MSG_C2C_SEMAPHORE, lambda m: self.start_turn())
        self.register_message_receive_handler(MSG_S2C_GRADS, self.handle_grads)
        self.register_message_receive_handler(MSG_S2C_FINISH, lambda m: self.finish())

    def start_turn(self):
        self.client.model.train()
        self._it = iter(self.client.train_data)
        self.forward_next()

    def forward_next(self):
        try:
            x, y = next(self._it)
        except StopIteration:
            self.run_eval()
            return
        self.client.optimizer.zero_grad(set_to_none=True)
        self.client.acts = self.client.model(x.to(self.client.device))
        m = Message(MSG_C2S_SEND_ACTS, self.rank, 0)
        m.add_params("activations", self.client.acts.detach().cpu())
        m.add_params("labels", y)
        self.send_message(m)

    def handle_grads(self, msg):
        self.client.acts.backward(msg.get("grads").to(self.client.device))
        self.client.optimizer.step()
        self.forward_next()

    def run_eval(self):
        self.send_message(Message(MSG_C2S_VALIDATION_MODE, self.rank, 0))
        self.client.model.eval()
        with torch.no_grad():
            for x, y in (self.client.test_data or []):
                m = Message(MSG_C2S_SEND_ACTS, self.rank, 0)
                m.add_params("activations", self.client.model(x.to(self.client.device)).cpu())
                m.add_params("labels", y)
                self.send_message(m)
        self.send_message(Message(MSG_C2S_VALIDATION_OVER, self.rank, 0))
        self.turns_done += 1
        if self.rank == self.max_rank and self.turns_done >= self.epochs:
            self.send_message(Message(MSG_C2S_PROTOCOL_FINISHED, self.rank, 0))
            return
        self.send_message(Message(MSG_C2C_SEMAPHORE, self.rank, (self.rank % self.max_rank) + 1))


def SplitNN_distributed(args, process_id, worker_number, comm, device, dataset, model, model_trainer=None, **_):
    client_model, server_model = model
    backend = "LOOPBACK" if comm is not None else str(getattr(args, "backend", "TCP"))
    if process_id == 0:
        srv = SplitNNServer(server_model, worker_number - 1, device, args)
        mgr = SplitNNServerManager(args, srv, comm, 0, worker_number, backend)
        mgr.run()
        return {"history": srv.history, "server_model": srv.model}
    (_, _, _, _, _, train_local, test_local, _) = dataset[:8]
    cid = process_id - 1
    cl = SplitNNClient(client_model, train_local[cid], test_local.get(cid), device, args)
    mgr = SplitNNClientManager(args, cl, comm, process_id, worker_number, backend)
    if process_id == 1:
        mgr.start_turn()
    mgr.run()
