"""Cheetah: distributed (data-parallel) training of one model across the GPUs of a node or a
silo — ``fedml_amd.run_distributed()`` (the reference's ``run_distributed`` is an empty stub,
`python/fedml/__init__.py:277`; its only DDP usage is torch DDP inside hierarchical silos and the
centralized ImageNet example).

One process per GPU, ``torch.distributed`` over RCCL. The global training set is sharded by rank
(strided, like DistributedSampler with ``drop_last=False``), gradients are bucket-all-reduced
during backward (``FlatDDP``), the optimizer is one fused kernel, evaluation counts are
all-reduced. bf16 autocast is used for the forward/backward when ``compute_dtype: bf16``.
"""
import logging
import time

import torch
import torch.nn as nn

from ..parallel import comm
from .ddp import FlatDDP, FlatOptimizer


def shard_batches(data, rank, world):
    """Strided shard of an iterable of (x, y) batches: batch i goes to rank i % world."""
    for i, b in enumerate(data):
        if i % world == rank:
            yield b


class CheetahTrainer:
    def __init__(self, args, device, model, dataset, process_group=None):
        self.args = args
        self.device = torch.device(device)
        self.rank, self.world = comm.init_process_group(device=self.device if self.device.type == "cuda" else None)
        self.model = model.to(self.device)
        self.ddp = FlatDDP(self.model, self.device, process_group,
                           bucket_mb=float(getattr(args, "ddp_bucket_mb", 64.0)))
        opt = str(getattr(args, "client_optimizer", "sgd")).lower()
        self.opt = FlatOptimizer(self.ddp, opt, lr=float(args.learning_rate),
                                 momentum=float(getattr(args, "momentum", 0.0) or 0.0),
                                 weight_decay=float(getattr(args, "weight_decay", 0.0) or 0.0),
                                 amsgrad=(opt == "adam"))
        self.train_data = dataset[2]
        self.test_data = dataset[3]
        dt = str(getattr(args, "compute_dtype", "fp32"))
        self.autocast = self.device.type == "cuda" and dt in ("bf16", "bfloat16")
        self.crit = nn.CrossEntropyLoss()
        self.history = []

    def train_epoch(self, epoch):
        self.ddp.train()
        losses = []
        for x, y in shard_batches(self.train_data, self.rank, self.world):
            x, y = x.to(self.device, non_blocking=True), y.to(self.device, non_blocking=True)
            self.opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.autocast):
                loss = self.crit(self.ddp(x), y)
            loss.backward()
            self.ddp.finish_gradient_sync()
            self.opt.step()
            losses.append(loss.detach())
        return torch.stack(losses).mean() if losses else torch.zeros((), device=self.device)

    @torch.no_grad()
    def evaluate(self):
        self.ddp.eval()
        stats = torch.zeros(3, dtype=torch.float64, device=self.device)  # correct, loss_sum, n
        for x, y in shard_batches(self.test_data, self.rank, self.world):
            x, y = x.to(self.device), y.to(self.device)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.autocast):
                out = self.ddp(x).float()
            stats[0] += (out.argmax(1) == y).sum()
            stats[1] += nn.functional.cross_entropy(out, y, reduction="sum")
            stats[2] += y.numel()
        comm.all_reduce_flat(stats)
        n = max(1.0, float(stats[2]))
        return {"test_acc": float(stats[0]) / n, "test_loss": float(stats[1]) / n}

    def train(self):
        for ep in range(int(self.args.epochs)):
            t0 = time.time()
            loss = float(self.train_epoch(ep))
            rec = {"epoch": ep, "train_loss": loss, "epoch_time_s": time.time() - t0}
            freq = int(getattr(self.args, "frequency_of_the_test", 1) or 1)
            if ep % freq == 0 or ep == int(self.args.epochs) - 1:
                rec.update(self.evaluate())
            self.history.append(rec)
            if self.rank == 0:
                logging.info("cheetah epoch %d: %s", ep, rec)
        return self.history
