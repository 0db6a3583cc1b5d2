"""Semantic-segmentation training utilities for FedSeg (reference:
`mpi_p2p_mp/fedseg/utils.py:56-299`, `MyModelTrainer.py:11-162`).

* ``SegmentationLosses`` — CE / focal with ``ignore_index=255``.
* ``Evaluator`` — confusion matrix accumulated ON DEVICE (one ``bincount`` per batch instead of
  the reference's per-batch numpy copy); pixel accuracy, class accuracy, mIoU, FWIoU.
* ``LR_Scheduler`` — poly / cos / step schedules.
* ``Saver`` — run directory with checkpoints and ``best_pred.txt``.
"""
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..core.alg_frame.client_trainer import ClientTrainer


class SegmentationLosses:
    def __init__(self, size_average=True, batch_average=True, ignore_index=255):
        self.ignore_index = ignore_index
        self.size_average = size_average
        self.batch_average = batch_average

    def build_loss(self, mode="ce"):
        return {"ce": self.CrossEntropyLoss, "focal": self.FocalLoss}[mode]

    def CrossEntropyLoss(self, logit, target):
        loss = F.cross_entropy(logit, target.long(), ignore_index=self.ignore_index,
                               reduction="mean" if self.size_average else "sum")
        return loss / logit.shape[0] if self.batch_average and not self.size_average else loss

    def FocalLoss(self, logit, target, gamma=2, alpha=0.5):
        logpt = -F.cross_entropy(logit, target.long(), ignore_index=self.ignore_index,
                                 reduction="mean" if self.size_average else "sum")
        pt = torch.exp(logpt)
        loss = -((1 - pt) ** gamma) * alpha * logpt
        return loss / logit.shape[0] if self.batch_average and not self.size_average else loss


class Evaluator:
    def __init__(self, num_class, device=None):
        self.num_class = num_class
        self.confusion_matrix = torch.zeros(num_class, num_class, dtype=torch.int64, device=device)

    def add_batch(self, gt_image, pre_image):
        gt = gt_image.reshape(-1).to(self.confusion_matrix.device).long()
        pr = pre_image.reshape(-1).to(self.confusion_matrix.device).long()
        mask = (gt >= 0) & (gt < self.num_class)
        idx = self.num_class * gt[mask] + pr[mask]
        self.confusion_matrix += torch.bincount(idx, minlength=self.num_class ** 2).view(self.num_class,
                                                                                        self.num_class)

    def _cm(self):
        return self.confusion_matrix.double().cpu()

    def Pixel_Accuracy(self):
        cm = self._cm()
        return float(torch.diagonal(cm).sum() / cm.sum().clamp_min(1))

    def Pixel_Accuracy_Class(self):
        cm = self._cm()
        acc = torch.diagonal(cm) / cm.sum(1)
        return float(acc[~torch.isnan(acc)].mean())

    def Mean_Intersection_over_Union(self):
        cm = self._cm()
        iou = torch.diagonal(cm) / (cm.sum(1) + cm.sum(0) - torch.diagonal(cm))
        return float(iou[~torch.isnan(iou)].mean())

    def Frequency_Weighted_Intersection_over_Union(self):
        cm = self._cm()
        freq = cm.sum(1) / cm.sum().clamp_min(1)
        iou = torch.diagonal(cm) / (cm.sum(1) + cm.sum(0) - torch.diagonal(cm))
        m = freq > 0
        return float((freq[m] * iou[m]).sum())

    def reset(self):
        self.confusion_matrix.zero_()


class LR_Scheduler:
    """mode ∈ {poly, cos, step}: lr(T) for iteration T of ``num_epochs × iters_per_epoch``."""

    def __init__(self, mode, base_lr, num_epochs, iters_per_epoch=0, lr_step=0, warmup_epochs=0):
        self.mode, self.lr, self.lr_step = mode, base_lr, lr_step
        self.iters_per_epoch = iters_per_epoch
        self.N = num_epochs * iters_per_epoch
        self.warmup_iters = warmup_epochs * iters_per_epoch

    def __call__(self, optimizer, i, epoch):
        T = epoch * self.iters_per_epoch + i
        if self.mode == "cos":
            lr = 0.5 * self.lr * (1 + math.cos(1.0 * T / max(1, self.N) * math.pi))
        elif self.mode == "poly":
            lr = self.lr * pow((1 - 1.0 * T / max(1, self.N)), 0.9)
        elif self.mode == "step":
            lr = self.lr * (0.1 ** (epoch // max(1, self.lr_step)))
        else:
            raise NotImplementedError(self.mode)
        if self.warmup_iters > 0 and T < self.warmup_iters:
            lr = lr * 1.0 * T / self.warmup_iters
        optimizer.param_groups[0]["lr"] = lr
        for g in optimizer.param_groups[1:]:
            g["lr"] = lr * 10
        return lr


class Saver:
    def __init__(self, args):
        root = getattr(args, "run_dir", None) or os.path.join(getattr(args, "checkpoint_dir", "./run"),
                                                              str(getattr(args, "dataset", "seg")),
                                                              str(getattr(args, "model", "model")))
        os.makedirs(root, exist_ok=True)
        runs = sorted(int(d.split("_")[-1]) for d in os.listdir(root) if d.startswith("experiment_"))
        self.experiment_dir = os.path.join(root, f"experiment_{(runs[-1] + 1) if runs else 0}")
        os.makedirs(self.experiment_dir, exist_ok=True)
        self.args = args

    def save_checkpoint(self, state, is_best, filename="checkpoint.pt"):
        torch.save(state, os.path.join(self.experiment_dir, filename))
        if is_best:
            with open(os.path.join(self.experiment_dir, "best_pred.txt"), "w") as f:
                f.write(str(state.get("best_pred", "")))
            torch.save(state, os.path.join(self.experiment_dir, "model_best.pt"))

    def save_experiment_config(self):
        with open(os.path.join(self.experiment_dir, "parameters.txt"), "w") as f:
            for k, v in sorted(vars(self.args).items()):
                if isinstance(v, (int, float, str, bool)):
                    f.write(f"{k}:{v}\n")


class ModelTrainerSeg(ClientTrainer):
    """``backbone_freezed`` (reference MyModelTrainer.py:12-25): only ``encoder_decoder`` trains and travels;
    otherwise backbone at 1× and head at 10× the learning rate when the model exposes the split."""

    def _frozen(self):
        return bool(getattr(self.args, "backbone_freezed", False)) and hasattr(self.model, "encoder_decoder")

    def _payload_module(self):
        return self.model.encoder_decoder if self._frozen() else self.model

    def get_model_params(self):
        return {k: v.detach().cpu().clone() for k, v in self._payload_module().state_dict().items()}

    def set_model_params(self, model_parameters):
        self._payload_module().load_state_dict(model_parameters)

    def train(self, train_data, device, args=None):
        args = args or self.args
        model = self.model.to(device)
        model.train()
        crit = SegmentationLosses().build_loss(str(getattr(args, "loss_type", "ce")))
        lr = float(args.learning_rate)
        kw = dict(momentum=float(getattr(args, "momentum", 0.9) or 0.9),
                  weight_decay=float(getattr(args, "weight_decay", 5e-4) or 5e-4),
                  nesterov=bool(getattr(args, "nesterov", False)))
        if self._frozen():   # head only, at 10× (the scheduler scales group 0 → keep base lr × 10 there)
            for p in model.backbone.parameters():
                p.requires_grad_(False)
            opt = torch.optim.SGD([p for p in model.parameters() if p.requires_grad], lr=lr * 10, **kw)
            lr = lr * 10
        elif hasattr(model, "get_1x_lr_params"):
            opt = torch.optim.SGD([{"params": model.get_1x_lr_params(), "lr": lr},
                                   {"params": model.get_10x_lr_params(), "lr": lr * 10}], **kw)
        else:
            opt = torch.optim.SGD(model.parameters(), lr=lr, **kw)
        sched = LR_Scheduler(str(getattr(args, "lr_scheduler", "poly")), lr, int(args.epochs), max(1, len(train_data)))
        losses = []
        for ep in range(int(args.epochs)):
            for i, (x, y) in enumerate(train_data):
                sched(opt, i, ep)
                x, y = x.to(device), y.to(device)
                opt.zero_grad(set_to_none=True)
                loss = crit(model(x), y)
                loss.backward()
                opt.step()
                losses.append(loss.detach())
        if losses:
            self.last_loss = float(torch.stack(losses).mean())
        return getattr(self, "last_loss", None)

    @torch.no_grad()
    def test(self, test_data, device, args=None):
        model = self.model.to(device)
        model.eval()
        crit = SegmentationLosses().build_loss("ce")
        ev = Evaluator(int(getattr(model, "n_classes", 0) or getattr(args or self.args, "class_num", 21)), device)
        loss, nb = 0.0, 0
        for x, y in test_data:
            x, y = x.to(device), y.to(device)
            out = model(x)
            loss += float(crit(out, y))
            nb += 1
            ev.add_batch(y, out.argmax(1))
        return {"test_acc": ev.Pixel_Accuracy(), "test_acc_class": ev.Pixel_Accuracy_Class(),
                "test_mIoU": ev.Mean_Intersection_over_Union(),
                "test_FWIoU": ev.Frequency_Weighted_Intersection_over_Union(), "test_loss": loss / max(1, nb),
                "test_correct": int(torch.diagonal(ev.confusion_matrix).sum()),
                "test_total": int(ev.confusion_matrix.sum())}
