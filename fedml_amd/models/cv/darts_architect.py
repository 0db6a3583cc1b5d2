"""DARTS architecture step (reference: ``model/cv/darts/architect.py``, used by
``mpi_p2p_mp/fednas/FedNASTrainer.py:11-305`` with ``--unrolled``).

First order: α ← Adam(∇_α L_val(w, α)). Second order (unrolled): the validation loss is taken at the
weights one SGD step ahead, w' = w − η·(μ·m + ∇_w L_train(w, α) + λ·w), so

    ∇_α L_val(w', α) − η · ∇²_{α,w} L_train(w, α) · ∇_{w'} L_val(w', α)

with the Hessian-vector product by central differences at w ± R·v, R = 0.01 / ‖v‖ (exactly the
reference's approximation). Written with ``torch.func.functional_call`` on the live module: no model
copy per step (the reference deep-copies the network for the unrolled model), BatchNorm buffers are
cloned so the extra forward passes never move the running statistics."""
import torch
import torch.nn as nn
from torch.func import functional_call


def _grad(loss, params):
    """autograd.grad with zeros for parameters the graph does not use (e.g. unused α of a cell type)."""
    gs = torch.autograd.grad(loss, params, allow_unused=True)
    return [torch.zeros_like(p) if g is None else g for p, g in zip(params, gs)]


class Architect:
    def __init__(self, model: nn.Module, args):
        self.model = model
        self.momentum = float(getattr(args, "momentum", 0.9) or 0.9)
        self.wd = float(getattr(args, "weight_decay", 3e-4) or 3e-4)
        self.crit = nn.CrossEntropyLoss()
        self.r = float(getattr(args, "arch_hvp_r", 0.01) or 0.01)   # reference: r = 1e-2
        self.optimizer = torch.optim.Adam(model.arch_parameters(), lr=float(getattr(args, "arch_learning_rate", 3e-4)),
                                          betas=(0.5, 0.999),
                                          weight_decay=float(getattr(args, "arch_weight_decay", 1e-3)))

    def _split(self):
        arch = {id(p) for p in self.model.arch_parameters()}
        W = {n: p for n, p in self.model.named_parameters() if id(p) not in arch}
        A = {n: p for n, p in self.model.named_parameters() if id(p) in arch}
        return W, A

    def _loss(self, W, A, x, y):
        bufs = {n: b.clone() for n, b in self.model.named_buffers()}
        return self.crit(functional_call(self.model, {**W, **A, **bufs}, (x,)), y)

    def step(self, x_train, y_train, x_val, y_val, eta, network_optimizer=None, unrolled=True):
        self.optimizer.zero_grad(set_to_none=True)
        if unrolled:
            self.unrolled_grads(x_train, y_train, x_val, y_val, eta, network_optimizer)
        else:
            W, A = self._split()
            grads = _grad(self._loss({n: p.detach() for n, p in W.items()}, A, x_val, y_val), list(A.values()))
            for p, g in zip(A.values(), grads):
                p.grad = g
        self.optimizer.step()

    def unrolled_grads(self, x_train, y_train, x_val, y_val, eta, network_optimizer=None):
        """Sets α.grad to the second-order (unrolled) architecture gradient; returns it."""
        W, A = self._split()
        A_det = {n: p.detach() for n, p in A.items()}
        Wd = {n: p.detach().requires_grad_(True) for n, p in W.items()}
        gW = _grad(self._loss(Wd, A_det, x_train, y_train), list(Wd.values()))
        Wu = {}
        for (n, p), g in zip(W.items(), gW):
            mom = 0.0
            if network_optimizer is not None:
                st = network_optimizer.state.get(p, {})
                if st.get("momentum_buffer") is not None:
                    mom = st["momentum_buffer"] * self.momentum
            Wu[n] = (p.detach() - eta * (mom + g + self.wd * p.detach())).requires_grad_(True)
        Lv = self._loss(Wu, A, x_val, y_val)
        gs = _grad(Lv, list(A.values()) + list(Wu.values()))
        dA, v = gs[:len(A)], gs[len(A):]
        R = self.r / torch.cat([t.reshape(-1) for t in v]).norm().clamp_min(1e-12)
        Wp = {n: (p.detach() + R * t) for (n, p), t in zip(W.items(), v)}
        Wm = {n: (p.detach() - R * t) for (n, p), t in zip(W.items(), v)}
        gp = _grad(self._loss(Wp, A, x_train, y_train), list(A.values()))
        gm = _grad(self._loss(Wm, A, x_train, y_train), list(A.values()))
        out = []
        for p, da, a_, b_ in zip(A.values(), dA, gp, gm):
            p.grad = da - eta * (a_ - b_) / (2 * R)
            out.append(p.grad)
        return out
