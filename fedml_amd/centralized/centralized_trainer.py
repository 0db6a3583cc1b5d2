"""Centralised training baseline (reference: `centralized/centralized_trainer.py:13-164`): one model
over the merged federated dataset, SGD or AMSGrad-Adam, per-epoch evaluation. With
``data_parallel: 1`` (or a torchrun world > 1) it delegates to the Cheetah data-parallel trainer
(bucketed RCCL all-reduce overlapped with backward) instead of the reference's torch DDP wrapper."""
import logging
import os

import torch
import torch.nn as nn

from ..core.mlops import MLOpsMetrics
from ..trainers.factory import make_optimizer


class CentralizedTrainer:
    def __init__(self, dataset, model, device, args):
        (self.train_data_num_in_total, self.test_data_num_in_total, self.train_global, self.test_global,
         self.train_data_local_num_dict, self.train_data_local_dict, self.test_data_local_dict,
         self.class_num) = dataset[:8]
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.args = args
        self.model = model.to(self.device)
        self.criterion = nn.CrossEntropyLoss()
        self.history = []
        world = int(os.environ.get("WORLD_SIZE", "1"))
        self.dp = int(getattr(args, "data_parallel", 0) or 0) == 1 or world > 1
        if self.dp:
            from ..distributed import CheetahTrainer
            self.cheetah = CheetahTrainer(args, self.device, self.model, dataset)
        else:
            self.optimizer = make_optimizer(self.model.parameters(), args)

    def train(self):
        if self.dp:
            self.history = self.cheetah.train()
            return self.history
        for epoch in range(int(self.args.epochs)):
            loss = self.train_impl(epoch)
            stats = {"epoch": epoch, "Train/Loss": loss}
            stats.update(self.eval_impl(epoch))
            self.history.append(stats)
            MLOpsMetrics.get_instance().log(stats, step=epoch)
        return self.history

    def train_impl(self, epoch_idx):
        self.model.train()
        losses = []
        for x, y in self.train_global:
            x, y = x.to(self.device, non_blocking=True), y.to(self.device, non_blocking=True)
            self.optimizer.zero_grad(set_to_none=True)
            loss = self.criterion(self.model(x), y)
            loss.backward()
            self.optimizer.step()
            losses.append(loss.detach())
        loss = float(torch.stack(losses).mean()) if losses else float("nan")
        logging.info("centralized epoch %d: train loss %.4f", epoch_idx, loss)
        return loss

    @torch.no_grad()
    def eval_impl(self, epoch_idx):
        out = {}
        for name, data in (("Train", self.train_global), ("Test", self.test_global)):
            if data is None:
                continue
            self.model.eval()
            correct = total = 0
            loss = 0.0
            for x, y in data:
                x, y = x.to(self.device), y.to(self.device)
                pred = self.model(x)
                loss += float(self.criterion(pred, y)) * y.numel()
                correct += int((pred.argmax(-1) == y).sum())
                total += y.numel()
            out[f"{name}/Acc"] = correct / max(1, total)
            out[f"{name}/Loss"] = loss / max(1, total)
        logging.info("centralized epoch %d: %s", epoch_idx, out)
        return out
