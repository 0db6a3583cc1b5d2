"""Classification trainer (reference: `single_process/fedavg/my_model_trainer_classification.py:11-159`).

Local SGD/Adam with cross-entropy; evaluation accumulates an on-device
confusion matrix (HIP kernel on GPU) instead of a per-batch ``.cpu().numpy()``,
from which accuracy and per-class recall/precision are derived (fork metrics)."""
import logging

import torch
import torch.nn as nn

from ..core.alg_frame.client_trainer import ClientTrainer
from ..core.alg_frame.functional import FunctionalTrainerMixin
from ..ops import confusion_matrix
from .factory import make_optimizer


class ModelTrainerCLS(ClientTrainer, FunctionalTrainerMixin):
    loss_name = "ce"

    def __init__(self, model, args=None):
        super().__init__(model, args)
        self.class_weight = None
        self.clip_grad_norm = None
        self.input_hook = None  # optional per-batch input transform on device (HS-FedAvg amplitude mixing)

    def get_model_params(self):
        return {k: v.detach().cpu().clone() for k, v in self.model.state_dict().items()}

    def set_model_params(self, model_parameters):
        self.model.load_state_dict(model_parameters)

    def _criterion(self, device):
        w = self.class_weight.to(device) if self.class_weight is not None else None
        return nn.CrossEntropyLoss(weight=w).to(device)

    def train(self, train_data, device, args=None):
        args = args or self.args
        model = self.model.to(device)
        model.train()
        criterion = self._criterion(device)
        optimizer = make_optimizer(model.parameters(), args)
        epoch_loss = []
        for epoch in range(int(args.epochs)):
            batch_loss = []
            for x, labels in train_data:
                x, labels = x.to(device, non_blocking=True), labels.to(device, non_blocking=True)
                if self.input_hook is not None:
                    x = self.input_hook(x)
                optimizer.zero_grad(set_to_none=True)
                loss = criterion(model(x), labels)
                loss.backward()
                if self.clip_grad_norm:
                    torch.nn.utils.clip_grad_norm_(model.parameters(), self.clip_grad_norm)
                optimizer.step()
                batch_loss.append(loss.detach())
            if batch_loss:
                epoch_loss.append(torch.stack(batch_loss).mean())
        if epoch_loss:
            self.last_loss = float(torch.stack(epoch_loss).mean())
            logging.debug("Client %s: local loss %.4f", self.id, self.last_loss)
        return self.last_loss if epoch_loss else None

    @torch.no_grad()
    def test(self, test_data, device, args=None):
        model = self.model.to(device)
        model.eval()
        metrics = {"test_correct": 0, "test_loss": 0.0, "test_total": 0}
        criterion = nn.CrossEntropyLoss(reduction="sum").to(device)
        cm = None
        loss_sum = torch.zeros((), device=device)
        for x, target in test_data:
            x, target = x.to(device), target.to(device)
            pred = model(x)
            if pred.dim() > 2:
                pred = pred.reshape(pred.shape[0], -1)
            loss_sum += criterion(pred.float(), target)
            c = confusion_matrix(pred.float().contiguous(), target)[0]
            cm = c if cm is None else cm + c
        if cm is not None:
            cm = cm.cpu()
            metrics["test_correct"] = int(torch.diagonal(cm).sum())
            metrics["test_total"] = int(cm.sum())
            metrics["test_loss"] = float(loss_sum)
            tp = torch.diagonal(cm).double()
            metrics["recall_per_class"] = (tp / cm.sum(1).clamp_min(1)).tolist()
            metrics["precision_per_class"] = (tp / cm.sum(0).clamp_min(1)).tolist()
            metrics["confusion_matrix"] = cm
            # the fork's per-class dicts over the classes present in the labels (simulation/common.class_rates)
            from ..simulation.common import class_rates
            metrics["test_recall"], metrics["test_precision"] = class_rates(tp, cm.sum(1), cm.sum(0))
        return metrics

    def test_on_the_server(self, train_data_local_dict, test_data_local_dict, device, args=None) -> bool:
        return False
