"""FedProx local trainer: CE + (μ/2)·‖w − w_global‖² (the reference's FedProx has no proximal term,
Appendix A #5; `mu` was read but unused)."""
import torch

from .classification import ModelTrainerCLS
from .factory import make_optimizer


class ModelTrainerFedProx(ModelTrainerCLS):
    def train(self, train_data, device, args=None):
        args = args or self.args
        mu = float(getattr(args, "fedprox_mu", getattr(args, "mu", 0.01)) or 0.0)
        model = self.model.to(device)
        model.train()
        global_params = [p.detach().clone() for p in model.parameters()]
        criterion = self._criterion(device)
        optimizer = make_optimizer(model.parameters(), args)
        losses = []
        for _ in range(int(args.epochs)):
            for x, y in train_data:
                x, y = x.to(device), y.to(device)
                optimizer.zero_grad(set_to_none=True)
                loss = criterion(model(x), y)
                if mu > 0:
                    prox = sum(((p - g) ** 2).sum() for p, g in zip(model.parameters(), global_params))
                    loss = loss + 0.5 * mu * prox
                loss.backward()
                optimizer.step()
                losses.append(loss.detach())
        self.last_loss = float(torch.stack(losses).mean()) if losses else None
        return self.last_loss
