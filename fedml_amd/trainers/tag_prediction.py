"""Multi-label tag prediction trainer (reference: `my_model_trainer_tag_prediction.py`):
BCELoss(sum) on sigmoid outputs, precision/recall at threshold 0.5."""
import torch
import torch.nn as nn

from .classification import ModelTrainerCLS
from .factory import make_optimizer


class ModelTrainerTAGPred(ModelTrainerCLS):
    loss_name = "bce_sum"

    def train(self, train_data, device, args=None):
        args = args or self.args
        model = self.model.to(device)
        model.train()
        criterion = nn.BCELoss(reduction="sum").to(device)
        optimizer = make_optimizer(model.parameters(), args)
        losses = []
        for _ in range(int(args.epochs)):
            for x, y in train_data:
                x, y = x.to(device), y.to(device).float()
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
        criterion = nn.BCELoss(reduction="sum").to(device)
        m = {"test_correct": 0.0, "test_loss": 0.0, "test_precision": 0.0, "test_recall": 0.0, "test_total": 0}
        for x, y in test_data:
            x, y = x.to(device), y.to(device).float()
            p = model(x)
            m["test_loss"] += float(criterion(p, y))
            pred = (p > 0.5).int()
            correct = pred.eq(y.int()).all(1).sum()
            tp = (pred * y.int()).sum(1).float()
            m["test_precision"] += float((tp / (pred.sum(1).float() + 1e-13)).sum())
            m["test_recall"] += float((tp / (y.sum(1) + 1e-13)).sum())
            m["test_correct"] += float(correct)
            m["test_total"] += y.size(0)
        return m
