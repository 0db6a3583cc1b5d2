"""Vertical FL, sequential (reference: `single_process/classical_vertical_fl/{vfl,party_models,
vfl_fixture}.py`): party A (guest) owns labels, other parties (hosts) own feature slices; per
batch hosts send partial logits ``U_k = dense_k(local_k(X_k))``, the guest sums them with its
own, computes BCE-with-logits and returns the common gradient ``∂L/∂U`` that every party
back-propagates locally. Parties are torch modules on the compute device (the reference
round-trips through numpy every batch)."""
import logging

import numpy as np
import torch
import torch.nn as nn

from ....models.finance.vfl_models import DenseModel, LocalModel
from ....utils.metrics import binary_prf, roc_auc


class _PartyBase:
    def __init__(self, local_model, bias, lr, device):
        self.localModel = local_model.to(device)
        out = getattr(local_model, "output_dim", None) or local_model.classifier[0].out_features
        self.dense_model = DenseModel(out, 1, bias=bias).to(device)
        self.device = device
        self.opt = torch.optim.SGD(list(self.localModel.parameters()) + list(self.dense_model.parameters()), lr=lr,
                                   momentum=0.9, weight_decay=0.01)

    def set_dense_model(self, dense_model):
        self.dense_model = dense_model.to(self.device)

    def _forward(self, X):
        return self.dense_model(self.localModel(X.to(self.device).float()))


class VFLGuestModel(_PartyBase):
    def __init__(self, local_model, lr=0.01, device="cpu"):
        super().__init__(local_model, True, lr, device)
        self.criterion = nn.BCEWithLogitsLoss()
        self.components = []

    def set_batch(self, X, y, global_step):
        self.X, self.y, self.current_global_step = X, y, global_step

    def receive_components(self, component_list):
        self.components.extend(component_list)

    def fit(self):
        own = self._forward(self.X)
        U = (own.detach() + sum(c.to(self.device) for c in self.components)).requires_grad_(True)
        loss = self.criterion(U, self.y.to(self.device).float().reshape(U.shape))
        (g,) = torch.autograd.grad(loss, U)
        self.opt.zero_grad(set_to_none=True)
        own.backward(g)
        self.opt.step()
        self.top_grads, self.loss = g.detach(), float(loss.detach())
        self.components = []

    def send_gradients(self):
        return self.top_grads

    def get_loss(self):
        return self.loss

    @torch.no_grad()
    def predict(self, X, component_list):
        U = self._forward(X) + sum(c.to(self.device) for c in component_list)
        return torch.sigmoid(U.sum(1))


class VFLHostModel(_PartyBase):
    def __init__(self, local_model, lr=0.01, device="cpu"):
        super().__init__(local_model, False, lr, device)

    def set_batch(self, X, global_step):
        self.X, self.current_global_step = X, global_step

    def send_components(self):
        self.opt.zero_grad(set_to_none=True)
        self._U = self._forward(self.X)
        return self._U.detach()

    def receive_gradients(self, gradients):
        self._U.backward(gradients.to(self.device))
        self.opt.step()

    @torch.no_grad()
    def predict(self, X):
        return self._forward(X)


class VerticalMultiplePartyLogisticRegressionFederatedLearning:
    def __init__(self, party_A, main_party_id="_main"):
        self.party_a = party_A
        self.main_party_id = main_party_id
        self.party_dict = {}

    def get_main_party_id(self):
        return self.main_party_id

    def add_party(self, *, id, party_model):
        self.party_dict[id] = party_model

    def fit(self, X_A, y, party_X_dict, global_step):
        self.party_a.set_batch(X_A, y, global_step)
        for k, X in party_X_dict.items():
            self.party_dict[k].set_batch(X, global_step)
        self.party_a.receive_components([p.send_components() for p in self.party_dict.values()])
        self.party_a.fit()
        g = self.party_a.send_gradients()
        for p in self.party_dict.values():
            p.receive_gradients(g)
        return self.party_a.get_loss()

    def predict(self, X_A, party_X_dict):
        return self.party_a.predict(X_A, [self.party_dict[k].predict(X) for k, X in party_X_dict.items()])


class FederatedLearningFixture:
    def __init__(self, federated_learning):
        self.federated_learning = federated_learning
        self.history = []

    def fit(self, train_data, test_data, epochs=50, batch_size=-1, recording_period=30):
        main = self.federated_learning.get_main_party_id()
        Xa, y = train_data[main]["X"], train_data[main]["Y"]
        Xa_t, y_t = test_data[main]["X"], test_data[main]["Y"]
        N = Xa.shape[0]
        bs = N if batch_size <= 0 else batch_size
        n_batches = (N + bs - 1) // bs
        step, losses = -1, []
        for ep in range(epochs):
            for b in range(n_batches):
                step += 1
                sl = slice(b * bs, (b + 1) * bs)
                parts = {k: X[sl] for k, X in train_data["party_list"].items()}
                losses.append(self.federated_learning.fit(Xa[sl], y[sl], parts, step))
                if (step + 1) % recording_period == 0:
                    self.history.append(self.evaluate(Xa_t, y_t, test_data["party_list"], ep, b, np.mean(losses)))
                    losses = []
        return self.history

    def evaluate(self, Xa_t, y_t, parts, ep=0, b=0, loss=float("nan")):
        prob = self.federated_learning.predict(Xa_t, parts).cpu()
        yt = torch.as_tensor(y_t).reshape(-1).float()
        pred = (prob > 0.5).float()
        p, r, f = binary_prf(pred, yt)
        stats = {"epoch": ep, "batch": b, "loss": float(loss), "acc": float((pred == yt).float().mean()),
                 "auc": roc_auc(prob, yt), "precision": p, "recall": r, "f1": f}
        logging.info("VFL: %s", stats)
        return stats


class VFLAPI:
    """SP entry: ``dataset = (train_parts, y_train, test_parts, y_test)`` (``data.vertical``); party 0
    is the guest. ``model``: optional list of per-party local models."""

    def __init__(self, args, device, dataset, model=None, model_trainer=None):
        self.args = args
        tr, ytr, te, yte = dataset[:4]
        dev = device or torch.device("cpu")
        hidden = int(getattr(args, "vfl_hidden_dim", 10))
        lr = float(getattr(args, "learning_rate", 0.01))
        locals_ = model if isinstance(model, (list, tuple)) else [LocalModel(p.shape[1], hidden) for p in tr]
        guest = VFLGuestModel(locals_[0], lr, dev)
        self.fl = VerticalMultiplePartyLogisticRegressionFederatedLearning(guest)
        for k in range(1, len(tr)):
            self.fl.add_party(id=f"party_{k}", party_model=VFLHostModel(locals_[k], lr, dev))
        self.train_data = {"_main": {"X": tr[0], "Y": ytr}, "party_list": {f"party_{k}": tr[k] for k in range(1, len(tr))}}
        self.test_data = {"_main": {"X": te[0], "Y": yte}, "party_list": {f"party_{k}": te[k] for k in range(1, len(te))}}
        self.fixture = FederatedLearningFixture(self.fl)

    def train(self):
        hist = self.fixture.fit(self.train_data, self.test_data, epochs=int(getattr(self.args, "comm_round", 10)),
                                batch_size=int(self.args.batch_size),
                                recording_period=int(getattr(self.args, "frequency_of_the_test", 30) or 30))
        final = self.fixture.evaluate(self.test_data["_main"]["X"], self.test_data["_main"]["Y"],
                                      self.test_data["party_list"])
        return {"history": hist, "final": final}
