"""Classical vertical FL over message passing (reference: `mpi_p2p_mp/classical_vertical_fl/*`).

Rank 0 is the guest (labels + its own feature slice), ranks 1..N are hosts (feature slices).
Per mini-batch: every host sends the partial logits of its slice (C2S_LOGITS); the guest adds
its own, computes BCE-with-logits, back-propagates through its classifier + extractor, and
returns ``∂L/∂logits`` (S2C_GRADIENT) — identical for every party because logits add — which
each host pushes through its own model. Test logits ride along every ``frequency_of_the_test``
steps so the guest can report accuracy / AUC on the joint model.

``dataset`` = ``(train_parts, y_train, test_parts, y_test)`` as from ``data.vertical``;
``model`` = list of ``(feature_extractor, classifier)`` per party.
"""
import logging

import torch
import torch.nn as nn

from ...core.distributed import ClientManager, Message, ServerManager
from ...utils.metrics import roc_auc as _auc

MSG_S2C_INIT_CONFIG = 1
MSG_S2C_GRADIENT = 2
MSG_C2S_LOGITS = 3
MSG_S2C_FINISH = 4


class _Party:
    def __init__(self, fe, clf, device, args):
        self.fe, self.clf = fe.to(device), clf.to(device)
        lr = float(getattr(args, "learning_rate", 0.01))
        self.opt = torch.optim.SGD(list(fe.parameters()) + list(clf.parameters()), lr=lr, momentum=0.9,
                                   weight_decay=0.01)
        self.device = device

    def logits(self, x):
        return self.clf(self.fe(x.to(self.device)))


class GuestTrainer(_Party):
    def __init__(self, n_hosts, X, y, Xt, yt, fe, clf, device, args):
        super().__init__(fe, clf, device, args)
        self.n_hosts = n_hosts
        self.X, self.y, self.Xt, self.yt = X, y, Xt, yt
        self.bs = int(args.batch_size)
        self.n_batches = (len(X) + self.bs - 1) // self.bs
        self.host_train, self.host_test = {}, {}
        self.crit = nn.BCEWithLogitsLoss()
        self.loss_list, self.history = [], []

    def add_client_local_result(self, idx, train_logits, test_logits):
        self.host_train[idx] = train_logits
        if test_logits is not None:
            self.host_test[idx] = test_logits

    def all_received(self):
        return len(self.host_train) == self.n_hosts

    def train(self, step):
        b = step % self.n_batches
        x = self.X[b * self.bs:(b + 1) * self.bs]
        y = self.y[b * self.bs:(b + 1) * self.bs].to(self.device).reshape(-1, 1)
        own = self.logits(x)
        total_host = sum(self.host_train[k].to(self.device) for k in sorted(self.host_train))
        z = (own.detach() + total_host).requires_grad_(True)
        loss = self.crit(z, y)
        (g,) = torch.autograd.grad(loss, z)
        self.opt.zero_grad(set_to_none=True)
        own.backward(g)
        self.opt.step()
        self.loss_list.append(float(loss))
        self.host_train.clear()
        return g.detach().cpu()

    @torch.no_grad()
    def test(self, step):
        if len(self.host_test) < self.n_hosts:
            return None
        z = self.logits(self.Xt).cpu() + sum(self.host_test[k] for k in sorted(self.host_test))
        p = torch.sigmoid(z).reshape(-1)
        acc = float(((p > 0.5).float() == self.yt).float().mean())
        stats = {"step": step, "test_acc": acc, "test_auc": _auc(p, self.yt),
                 "train_loss": sum(self.loss_list[-self.n_batches:]) / max(1, len(self.loss_list[-self.n_batches:]))}
        self.history.append(stats)
        self.host_test.clear()
        logging.info("VFL guest: %s", stats)
        return stats


class HostTrainer(_Party):
    def __init__(self, X, Xt, fe, clf, device, args):
        super().__init__(fe, clf, device, args)
        self.X, self.Xt = X, Xt
        self.bs = int(args.batch_size)
        self.n_batches = (len(X) + self.bs - 1) // self.bs
        self._out = None

    def computer_logits(self, step, with_test):
        b = step % self.n_batches
        self.opt.zero_grad(set_to_none=True)
        self._out = self.logits(self.X[b * self.bs:(b + 1) * self.bs])
        test = None
        if with_test:
            with torch.no_grad():
                test = self.logits(self.Xt).cpu()
        return self._out.detach().cpu(), test

    def update_model(self, grad):
        self._out.backward(grad.to(self.device))
        self.opt.step()


def _test_due(args, step, total):
    f = int(getattr(args, "frequency_of_the_test", 0) or 0)
    return step == total - 1 or (f > 0 and (step + 1) % f == 0)


class GuestManager(ServerManager):
    def __init__(self, args, trainer, comm, rank, size, backend):
        super().__init__(args, comm, rank, size, backend)
        self.trainer = trainer
        self.step = 0
        self.total = int(args.comm_round) * trainer.n_batches if getattr(args, "vfl_steps", None) is None \
            else int(args.vfl_steps)

    def register_message_receive_handlers(self):
        self.register_message_receive_handler(MSG_C2S_LOGITS, self.handle_logits)

    def send_init(self):
        for r in range(1, self.size):
            m = Message(MSG_S2C_INIT_CONFIG, 0, r)
            m.add_params("total_steps", self.total)
            self.send_message(m)

    def handle_logits(self, msg):
        self.trainer.add_client_local_result(msg.get_sender_id() - 1, msg.get("train_logits"),
                                             msg.get("test_logits"))
        if not self.trainer.all_received():
            return
        g = self.trainer.train(self.step)
        if _test_due(self.args, self.step, self.total):
            self.trainer.test(self.step)
        self.step += 1
        for r in range(1, self.size):
            m = Message(MSG_S2C_GRADIENT, 0, r)
            m.add_params("gradient", g)
            self.send_message(m)
        if self.step >= self.total:
            for r in range(1, self.size):
                self.send_message(Message(MSG_S2C_FINISH, 0, r))
            self.finish()


class HostManager(ClientManager):
    def __init__(self, args, trainer, comm, rank, size, backend):
        super().__init__(args, comm, rank, size, backend)
        self.trainer = trainer
        self.step = 0
        self.total = 0

    def register_message_receive_handlers(self):
        self.register_message_receive_handler(MSG_S2C_INIT_CONFIG, self.handle_init)
        self.register_message_receive_handler(MSG_S2C_GRADIENT, self.handle_grad)
        self.register_message_receive_handler(MSG_S2C_FINISH, lambda m: self.finish())

    def handle_init(self, msg):
        self.total = int(msg.get("total_steps"))
        self.send_logits()

    def send_logits(self):
        tr, te = self.trainer.computer_logits(self.step, _test_due(self.args, self.step, self.total))
        m = Message(MSG_C2S_LOGITS, self.rank, 0)
        m.add_params("train_logits", tr)
        m.add_params("test_logits", te)
        self.send_message(m)

    def handle_grad(self, msg):
        self.trainer.update_model(msg.get("gradient"))
        self.step += 1
        if self.step < self.total:
            self.send_logits()


def FedML_VFL_distributed(args, process_id, worker_number, comm, device, dataset, model, model_trainer=None, **_):
    train_parts, y_train, test_parts, y_test = dataset[:4]
    backend = "LOOPBACK" if comm is not None else str(getattr(args, "backend", "TCP"))
    fe, clf = model[process_id]
    if process_id == 0:
        t = GuestTrainer(worker_number - 1, train_parts[0], y_train, test_parts[0], y_test, fe, clf, device, args)
        mgr = GuestManager(args, t, comm, 0, worker_number, backend)
        mgr.send_init()
        mgr.run()
        return {"history": t.history, "loss": t.loss_list}
    t = HostTrainer(train_parts[process_id], test_parts[process_id], fe, clf, device, args)
    mgr = HostManager(args, t, comm, process_id, worker_number, backend)
    mgr.run()
