"""Next-word-prediction trainer (reference: `my_model_trainer_nwp.py`): CE with ignore_index=0
(padding), accuracy over non-padding tokens."""
import torch
import torch.nn as nn

from .classification import ModelTrainerCLS
from .factory import make_optimizer


class ModelTrainerNWP(ModelTrainerCLS):
    loss_name = "nwp_ce"

    def train(self, train_data, device, args=None):
        args = args or self.args
        model = self.model.to(device)
        model.train()
        criterion = nn.CrossEntropyLoss(ignore_index=0).to(device)
        optimizer = make_optimizer(model.parameters(), args)
        losses = []
        for _ in range(int(args.epochs)):
            for x, y in train_data:
                x, y = x.to(device), y.to(device)
                optimizer.zero_grad(set_to_none=True)
                loss = criterion(model(x), y)
                loss.backward()
                optimizer.step()
                losses.append(loss.detach())
        self.last_loss = float(torch.stack(losses).mean()) if losses else None
        return self.last_loss

    @torch.no_grad()
    def test(self, test_data, device, args=None):
        model = self.model.to(device)
        model.eval()
        criterion = nn.CrossEntropyLoss(ignore_index=0, reduction="sum").to(device)
        correct = torch.zeros((), device=device)
        total = torch.zeros((), device=device)
        loss = torch.zeros((), device=device)
        for x, y in test_data:
            x, y = x.to(device), y.to(device)
            pred = model(x)
            loss += criterion(pred, y)
            pi = pred.argmax(1)
            mask = y != 0
            correct += (pi.eq(y) & mask).sum()
            total += mask.sum()
        return {"test_correct": int(correct), "test_loss": float(loss), "test_total": int(total)}
