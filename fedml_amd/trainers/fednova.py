"""FedNova local optimizer + trainer (reference: `single_process/fednova/fednova.py:12-169`,
`client.py:50-112`; Wang et al. 2020).

SGD with optional momentum / Nesterov / weight decay and a proximal term ``μ(w − w₀)``;
tracks the local normalising constant ``a_i`` (Σ of the momentum-geometric step weights,
or the prox-damped count) that FedNova divides the client's cumulative update by. The
server-side normalised average is ``core.server_update.fednova_aggregate``.
"""
import torch

from .classification import ModelTrainerCLS


class FedNovaOptimizer(torch.optim.Optimizer):
    def __init__(self, params, lr, ratio=1.0, gmf=0.0, mu=0.0, momentum=0.0, dampening=0.0, weight_decay=0.0,
                 nesterov=False):
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                      nesterov=nesterov))
        self.gmf, self.mu, self.ratio, self.momentum = gmf, mu, ratio, momentum
        self.local_normalizing_vec = 0.0
        self.local_counter = 0.0
        self.local_steps = 0

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        lr = None
        for g in self.param_groups:
            lr = g["lr"]
            for p in g["params"]:
                if p.grad is None:
                    continue
                d = p.grad
                if g["weight_decay"]:
                    d = d.add(p, alpha=g["weight_decay"])
                st = self.state[p]
                if "old_init" not in st:
                    st["old_init"] = p.detach().clone()
                if g["momentum"]:
                    if "momentum_buffer" not in st:
                        buf = st["momentum_buffer"] = d.detach().clone()
                    else:
                        buf = st["momentum_buffer"]
                        buf.mul_(g["momentum"]).add_(d, alpha=1 - g["dampening"])
                    d = d.add(buf, alpha=g["momentum"]) if g["nesterov"] else buf
                if self.mu:
                    prox = p.detach() - st["old_init"]
                    if g["momentum"] and not g["nesterov"]:
                        # the reference adds in place (fednova.py:140 `d_p.add_(self.mu, …)`) and d_p IS the
                        # momentum buffer here, so the proximal term accumulates in the buffer
                        buf.add_(prox, alpha=self.mu)
                    else:
                        d = d.add(prox, alpha=self.mu)
                if "cum_grad" not in st:
                    st["cum_grad"] = d.detach().clone().mul_(lr)
                else:
                    st["cum_grad"].add_(d, alpha=lr)
                p.add_(d, alpha=-lr)
        if self.momentum:
            self.local_counter = self.local_counter * self.momentum + 1
            self.local_normalizing_vec += self.local_counter
        etamu = (lr or 0.0) * self.mu
        if etamu:
            self.local_normalizing_vec *= 1 - etamu
            self.local_normalizing_vec += 1
        if not self.momentum and not etamu:
            self.local_normalizing_vec += 1
        self.local_steps += 1
        return loss

    def tau_eff(self):
        return self.local_steps * self.ratio if self.mu else self.local_normalizing_vec * self.ratio


class ModelTrainerFedNova(ModelTrainerCLS):
    """``train`` returns the trainer state needed by the server: (a_i, τ_eff_i)."""

    def train(self, train_data, device, args=None, ratio=1.0):
        args = args or self.args
        model = self.model.to(device)
        model.train()
        crit = self._criterion(device)
        opt = FedNovaOptimizer(model.parameters(), lr=float(args.learning_rate), ratio=float(ratio),
                               gmf=float(getattr(args, "gmf", 0.0) or 0.0), mu=float(getattr(args, "mu", 0.0) or 0.0),
                               momentum=float(getattr(args, "momentum", 0.0) or 0.0),
                               dampening=float(getattr(args, "dampening", 0.0) or 0.0),
                               weight_decay=float(getattr(args, "wd", getattr(args, "weight_decay", 0.0)) or 0.0),
                               nesterov=bool(getattr(args, "nesterov", False)))
        losses = []
        for _ in range(int(args.epochs)):
            for x, y in train_data:
                x, y = x.to(device), y.to(device)
                opt.zero_grad(set_to_none=True)
                loss = crit(model(x), y)
                loss.backward()
                opt.step()
                losses.append(loss.detach())
        self.last_loss = float(torch.stack(losses).mean()) if losses else None
        self.a_i = max(opt.local_normalizing_vec, 1e-12)
        self.tau_eff_i = opt.tau_eff()
        return self.last_loss
