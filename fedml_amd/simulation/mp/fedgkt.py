"""FedGKT — group knowledge transfer (reference: `mpi_p2p_mp/fedgkt/*`, He et al. 2020).

Clients train a small net (``ResNetClient``: returns ``(logits, features)``) with CE plus a
temperature-scaled KL term toward the server's per-batch logits, then upload — per local batch —
the extracted feature maps, their own logits and labels. The server trains the large trunk
(``ResNetServer``) on the pooled features with KL-to-client-logits + α·CE, and returns its logits
for every client batch. Feature maps travel as bf16 tensors in the pickle-free frame format (the
reference pickles float32 numpy dicts), halving the uplink.

``model`` is the pair ``(client_model, server_model)``.
"""
import logging

import torch
import torch.nn as nn
import torch.nn.functional as F

from ...core.distributed import ClientManager, Message, ServerManager
from ...data.client_data import ClientData

MSG_S2C_SYNC_TO_CLIENT = 1
MSG_C2S_SEND_FEATURE_AND_LOGITS = 2
MSG_S2C_FINISH = 3


class KLLoss(nn.Module):
    """KL(teacher ‖ student) at temperature T, scaled by T² (reference `fedgkt/utils.py` KL_Loss)."""

    def __init__(self, temperature=3.0):
        super().__init__()
        self.T = float(temperature)

    def forward(self, student_logits, teacher_logits):
        s = F.log_softmax(student_logits / self.T, dim=1)
        t = F.softmax(teacher_logits.float() / self.T, dim=1) + 1e-7
        return self.T * self.T * F.kl_div(s, t, reduction="batchmean")


def _opt(params, args, lr):
    if str(getattr(args, "optimizer", getattr(args, "client_optimizer", "sgd"))).lower() == "sgd":
        return torch.optim.SGD(params, lr=lr, momentum=0.9, nesterov=True,
                               weight_decay=float(getattr(args, "wd", getattr(args, "weight_decay", 5e-4)) or 5e-4))
    return torch.optim.Adam(params, lr=lr, weight_decay=1e-4, amsgrad=True)


class GKTClientTrainer:
    def __init__(self, client_index, train_data_local_dict, test_data_local_dict, train_data_local_num_dict, device,
                 client_model, args):
        self.client_index = client_index
        td = train_data_local_dict[client_index]
        # fixed batch order: server logits are keyed by batch index, so the KD targets must line up
        self.train_data = ClientData(td.x, td.y, td.batch_size) if isinstance(td, ClientData) else td
        self.test_data = test_data_local_dict.get(client_index)
        self.local_sample_number = train_data_local_num_dict[client_index]
        self.device = device
        self.args = args
        self.model = client_model.to(device)
        self.optimizer = _opt(self.model.parameters(), args, float(args.learning_rate))
        self.ce = nn.CrossEntropyLoss()
        self.kl = KLLoss(float(getattr(args, "temperature", 3.0)))
        self.server_logits = {}
        self.feat_dtype = torch.bfloat16 if str(getattr(args, "gkt_feature_dtype", "bf16")) == "bf16" else torch.float32

    def update_large_model_logits(self, logits):
        self.server_logits = logits

    def train(self):
        args_ = self.args
        alpha = float(getattr(args_, "alpha", 1.0))
        if int(getattr(args_, "whether_training_on_client", 1)) == 1:
            self.model.train()
            for _ in range(int(getattr(args_, "epochs_client", getattr(args_, "epochs", 1)))):
                for b, (x, y) in enumerate(self.train_data):
                    x, y = x.to(self.device), y.to(self.device)
                    logits, _ = self.model(x)
                    loss = self.ce(logits, y)
                    if str(b) in self.server_logits:
                        loss = loss + alpha * self.kl(logits, self.server_logits[str(b)].to(self.device))
                    self.optimizer.zero_grad(set_to_none=True)
                    loss.backward()
                    self.optimizer.step()
        self.model.eval()
        feats, logits_d, labels = {}, {}, {}
        feats_t, labels_t = {}, {}
        with torch.no_grad():
            for b, (x, y) in enumerate(self.train_data):
                lg, f = self.model(x.to(self.device))
                feats[str(b)] = f.to(self.feat_dtype).cpu()
                logits_d[str(b)] = lg.float().cpu()
                labels[str(b)] = y.cpu()
            if self.test_data is not None:
                for b, (x, y) in enumerate(self.test_data):
                    _, f = self.model(x.to(self.device))
                    feats_t[str(b)] = f.to(self.feat_dtype).cpu()
                    labels_t[str(b)] = y.cpu()
        return feats, logits_d, labels, feats_t, labels_t


class GKTServerTrainer:
    def __init__(self, client_num, device, server_model, args):
        self.client_num = client_num
        self.device = device
        self.args = args
        self.model = server_model.to(device)
        self.optimizer = _opt(self.model.parameters(), args, float(getattr(args, "server_lr", args.learning_rate)))
        self.ce = nn.CrossEntropyLoss()
        self.kl = KLLoss(float(getattr(args, "temperature", 3.0)))
        self.feats, self.logits, self.labels, self.feats_t, self.labels_t = {}, {}, {}, {}, {}
        self.flags = {i: False for i in range(client_num)}
        self.server_logits = {}
        self.history = []

    def add_local_trained_result(self, idx, feats, logits, labels, feats_t, labels_t):
        self.feats[idx], self.logits[idx], self.labels[idx] = feats, logits, labels
        self.feats_t[idx], self.labels_t[idx] = feats_t, labels_t
        self.flags[idx] = True

    def check_whether_all_receive(self):
        if not all(self.flags.values()):
            return False
        self.flags = {i: False for i in self.flags}
        return True

    def get_global_logits(self, idx):
        return self.server_logits.get(idx, {})

    def train(self, round_idx):
        alpha = float(getattr(self.args, "alpha", 1.0))
        self.model.train()
        epochs = int(getattr(self.args, "epochs_server", 1))
        losses = []
        for _ in range(epochs):
            for idx in sorted(self.feats):
                for b in self.feats[idx]:
                    f = self.feats[idx][b].to(self.device).float()
                    y = self.labels[idx][b].to(self.device)
                    out = self.model(f)
                    if int(getattr(self.args, "whether_distill_on_the_server", 1)) == 1:
                        loss = self.kl(out, self.logits[idx][b].to(self.device)) + alpha * self.ce(out, y)
                    else:
                        loss = self.ce(out, y)
                    self.optimizer.zero_grad(set_to_none=True)
                    loss.backward()
                    self.optimizer.step()
                    losses.append(loss.detach())
        self.model.eval()
        with torch.no_grad():
            for idx in sorted(self.feats):
                self.server_logits[idx] = {b: self.model(f.to(self.device).float()).float().cpu()
                                           for b, f in self.feats[idx].items()}
        stats = {"round": round_idx, "train_loss": float(torch.stack(losses).mean()) if losses else None}
        stats.update(self.eval())
        self.history.append(stats)
        logging.info("FedGKT server: %s", stats)

    @torch.no_grad()
    def eval(self):
        correct = total = 0
        for idx in self.feats_t:
            for b, f in self.feats_t[idx].items():
                out = self.model(f.to(self.device).float())
                correct += int((out.argmax(1).cpu() == self.labels_t[idx][b]).sum())
                total += int(self.labels_t[idx][b].numel())
        return {"test_acc": correct / total if total else None}


class GKTServerManager(ServerManager):
    def __init__(self, args, trainer, comm, rank, size, backend):
        super().__init__(args, comm, rank, size, backend)
        self.trainer = trainer
        self.round_idx = 0
        self.round_num = int(args.comm_round)

    def register_message_receive_handlers(self):
        self.register_message_receive_handler(MSG_C2S_SEND_FEATURE_AND_LOGITS, self.handle_features)

    def handle_features(self, msg):
        s = msg.get_sender_id()
        self.trainer.add_local_trained_result(s - 1, msg.get("feature"), msg.get("logits"), msg.get("labels"),
                                              msg.get("feature_test"), msg.get("labels_test"))
        if not self.trainer.check_whether_all_receive():
            return
        self.trainer.train(self.round_idx)
        self.round_idx += 1
        done = self.round_idx >= self.round_num
        for r in range(1, self.size):
            m = Message(MSG_S2C_FINISH if done else MSG_S2C_SYNC_TO_CLIENT, 0, r)
            if not done:
                m.add_params("global_logits", self.trainer.get_global_logits(r - 1))
            self.send_message(m)
        if done:
            self.finish()


class GKTClientManager(ClientManager):
    def __init__(self, args, trainer, comm, rank, size, backend):
        super().__init__(args, comm, rank, size, backend)
        self.trainer = trainer

    def register_message_receive_handlers(self):
        self.register_message_receive_handler(MSG_S2C_SYNC_TO_CLIENT, self.handle_logits)
        self.register_message_receive_handler(MSG_S2C_FINISH, lambda m: self.finish())

    def handle_logits(self, msg):
        self.trainer.update_large_model_logits(msg.get("global_logits"))
        self.train_and_send()

    def train_and_send(self):
        f, lg, y, ft, yt = self.trainer.train()
        m = Message(MSG_C2S_SEND_FEATURE_AND_LOGITS, self.rank, 0)
        m.add_params("feature", f)
        m.add_params("logits", lg)
        m.add_params("labels", y)
        m.add_params("feature_test", ft)
        m.add_params("labels_test", yt)
        self.send_message(m)


def FedML_FedGKT_distributed(args, process_id, worker_number, comm, device, dataset, model, model_trainer=None,
                             **_):
    client_model, server_model = model
    backend = "LOOPBACK" if comm is not None else str(getattr(args, "backend", "TCP"))
    (_, _, _, _, train_num_dict, train_local, test_local, _) = dataset[:8]
    if process_id == 0:
        st = GKTServerTrainer(worker_number - 1, device, server_model, args)
        mgr = GKTServerManager(args, st, comm, 0, worker_number, backend)
        mgr.run()
        return {"history": st.history, "server_model": st.model}
    ct = GKTClientTrainer(process_id - 1, train_local, test_local, train_num_dict, device, client_model, args)
    mgr = GKTClientManager(args, ct, comm, process_id, worker_number, backend)
    mgr.train_and_send()
    mgr.run()
