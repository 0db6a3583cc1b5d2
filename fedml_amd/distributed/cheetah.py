"""Cheetah: distributed (data-parallel) training of one model across the GPUs of a node or a
silo — ``fedml_amd.run_distributed()``.

Reference: the reference's ``run_distributed`` is an empty stub (`python/fedml/__init__.py:277`); its only DDP
training is torch DDP inside hierarchical silos and the centralized ImageNet example
(`examples/centralized/main.py:504-511,597-603`: ``init_process_group("nccl")`` + ``DistributedDataParallel`` +
``DistributedSampler``), with the silo split of `data/data_loader_cross_silo.py:22-47`.

One process per GPU, ``torch.distributed`` over RCCL. Data follow ``DistributedSampler`` semantics
(``drop_last=False``): every epoch one permutation shared by all ranks (seed + epoch), padded by wrapping to a
multiple of the replica count, replica q takes ``order[q::Q]`` — so every replica runs the SAME number of steps
with the same batch sizes (the collectives of the last, ragged step still match on every rank) and one step of Q
replicas × b samples is one global batch of Q·b consecutive samples of the padded order.

Two executors:

* native (GPU, CIFAR ResNets that ``parallel.native_resnet.parse_resnet`` accepts): ``replicas_per_gpu`` = R
  data-parallel replicas of the model run as ONE client-batched native HIP step (``NativeResNetStep`` with
  C = R — the same kernels as the FL engine; per-replica BatchNorm, like per-rank BN under DDP). The R replica
  gradients are averaged on the device (``weighted_sum`` kernel), all-reduced across ranks as one flat buffer,
  and one fused optimizer kernel updates the master row, which is then broadcast to the R rows. BatchNorm running
  statistics follow replica 0 of rank 0 (torch DDP's ``broadcast_buffers``): they ride in the buffer slots of the
  same all-reduce (rank 0 contributes them, the other ranks zeros) — one collective per step.
* torch (anything else, CPU): ``FlatDDP`` — bucketed all-reduce overlapped with backward — and the fused flat
  optimizer; bf16 autocast when ``compute_dtype: bf16``.

R ranks × 1 replica and 1 rank × R replicas are the same computation (tests/test_cheetah*.py).
"""
import logging
import math
import time

import torch
import torch.nn as nn

from .. import ops
from ..parallel import comm
from .ddp import FlatDDP, FlatOptimizer


def shard_indices(n: int, replica: int, n_replicas: int, epoch: int = 0, shuffle: bool = False, seed: int = 0):
    """Sample indices of ``replica`` for one epoch, ``DistributedSampler(drop_last=False)`` semantics: the
    (optionally shuffled) order is padded by wrapping to a multiple of ``n_replicas``, replica q takes
    ``order[q::n_replicas]``. Every replica gets ⌈n / n_replicas⌉ indices."""
    if shuffle:
        g = torch.Generator()
        g.manual_seed(int(seed) * 1000003 + int(epoch))
        order = torch.randperm(n, generator=g)
    else:
        order = torch.arange(n)
    per = math.ceil(n / n_replicas)
    pad = per * n_replicas - n
    if pad:
        order = torch.cat([order, order[torch.arange(pad) % max(n, 1)]])
    return order[replica::n_replicas]


def shard_batches(data, rank, world, batch_size=None, epoch=0, shuffle=False, seed=0):
    """(x, y) batches of this rank's shard of ``data`` (a ``ClientData``-like object with ``.x`` / ``.y``, or a
    list of (x, y) batches): equal batch counts and sizes on every rank (``shard_indices``)."""
    from ..data.client_data import batches_to_client_data
    if not hasattr(data, "x"):
        data = batches_to_client_data(list(data), batch_size or 1)
    bs = int(batch_size or data.batch_size)
    idx = shard_indices(len(data.x), rank, world, epoch, shuffle, seed)
    for s in range(0, len(idx), bs):
        sel = idx[s:s + bs]
        yield data.x[sel], data.y[sel]


class CheetahTrainer:
    def __init__(self, args, device, model, dataset, process_group=None):
        from ..data.client_data import batches_to_client_data
        from ..utils import determinism
        self.args = args
        self.device = torch.device(device)
        self.det = determinism.enabled(args)
        if self.det:
            determinism.enable(args)
        self.rank, self.world = comm.init_process_group(device=self.device if self.device.type == "cuda" else None,
                                                        args=args)
        self.pg = process_group
        self.model = model.to(self.device)
        self.bs = int(getattr(args, "batch_size", 64))
        train, test = dataset[2], dataset[3]
        self.train_data = train if hasattr(train, "x") else batches_to_client_data(list(train), self.bs)
        self.test_data = test if (test is None or hasattr(test, "x")) else batches_to_client_data(list(test), self.bs)
        self.shuffle = bool(getattr(args, "shuffle", True))
        self.seed = int(getattr(args, "random_seed", 0) or 0)
        self.lr = float(args.learning_rate)
        self.momentum = float(getattr(args, "momentum", 0.0) or 0.0)
        self.wd = float(getattr(args, "weight_decay", 0.0) or 0.0)
        self.opt_name = str(getattr(args, "client_optimizer", "sgd")).lower()
        dt = str(getattr(args, "compute_dtype", "fp32") or "fp32")
        self.compute_dtype = torch.bfloat16 if (self.device.type == "cuda" and dt in ("bf16", "bfloat16")) else None
        self.crit = nn.CrossEntropyLoss()
        self.history = []
        self.samples_seen = 0
        self.native = None
        mode = str(getattr(args, "cheetah_exec", "auto") or "auto")
        if self.device.type == "cuda" and mode in ("auto", "native"):
            self._try_native(int(getattr(args, "replicas_per_gpu", 1) or 1), required=mode == "native")
        if self.native is None:
            self.R = 1
            self.ddp = FlatDDP(self.model, self.device, process_group,
                               bucket_mb=float(getattr(args, "ddp_bucket_mb", 64.0)))
            self.opt = FlatOptimizer(self.ddp, self.opt_name, lr=self.lr, momentum=self.momentum,
                                     weight_decay=self.wd, amsgrad=(self.opt_name == "adam"))
        logging.info("cheetah: rank %d/%d, %s executor, %d replica(s) per GPU", self.rank, self.world,
                     "native" if self.native is not None else "torch", self.R)

    # ------------------------------------------------------------------ native executor
    def _try_native(self, R, required):
        from ..core.arena import ParamLayout
        from ..parallel.native_resnet import NativeResNetStep, UnsupportedNative
        layout = ParamLayout.from_module(self.model)
        try:
            step = NativeResNetStep(self.model, layout, R, self.device, dtype=self.compute_dtype or torch.float32)
        except UnsupportedNative as e:
            if required:
                raise
            logging.info("cheetah: torch executor (%s)", e)
            return
        if self.compute_dtype is None:
            from ..ops import nn_ops
            nn_ops.set_f32_mma_mode(str(getattr(self.args, "fp32_mma", "exact") or "exact"))
        if self.det:
            step.enable_deterministic()
        self.native, self.layout, self.R = step, layout, R
        dev = self.device
        self.params = layout.alloc_stack(R, dev)
        self.grads = layout.alloc_stack(R, dev)
        flat = layout.flatten(self.model.state_dict(), device=dev)
        comm.broadcast_flat(flat, 0, self.pg)               # every rank starts from rank 0's weights
        ops.broadcast_rows_(self.params, flat)
        self.gsum = torch.zeros(1, layout.size, dtype=torch.float32, device=dev)
        self.tmask = layout.trainable_mask(dev).to(torch.bool)
        self.bmask = ~self.tmask                             # BN running statistics / counters (+ alignment pad)
        self.wmask = self.tmask.to(torch.float32) if self.wd else None
        self.mom = torch.zeros(1, layout.size, device=dev) if (self.opt_name == "sgd" and self.momentum) else None
        if self.opt_name != "sgd":
            self.m1 = torch.zeros(1, layout.size, device=dev)
            self.m2 = torch.zeros(1, layout.size, device=dev)
            self.vmax = torch.zeros(1, layout.size, device=dev) if self.opt_name == "adam" else None
        self.t = 0
        self.rep_w = torch.full((R,), 1.0 / (R * self.world), dtype=torch.float32, device=dev)
        self.active = torch.ones(R, dtype=torch.float32, device=dev)
        self._nimg = {}
        self.x_dev = self.train_data.x.to(dev, non_blocking=True)
        self.y_dev = self.train_data.y.to(dev, non_blocking=True)

    def _native_step(self, idx):
        """idx [R, b] sample indices (one row per local replica)."""
        R, b = idx.shape
        x = self.x_dev[idx.reshape(-1)].view(R, b, *self.x_dev.shape[1:]).float()
        y = self.y_dev[idx.reshape(-1)].view(R, b).long()
        nimg = self._nimg.get(b)
        if nimg is None:
            nimg = self._nimg[b] = (torch.full((R,), b, dtype=torch.int32, device=self.device),
                                    torch.full((R, b), 1.0 / b, dtype=torch.float32, device=self.device))
        self.grads.zero_()
        loss = self.native.step(self.params, self.grads, x, y, nimg[1], self.active, nimg=nimg[0])
        g = self.gsum[0]
        ops.weighted_sum(self.grads, self.rep_w, out=g)                # mean over local replicas (÷ R·world)
        # rank 0 contributes replica 0's BN running statistics in the buffer slots: after the SUM all-reduce every
        # rank holds them (torch DDP broadcast_buffers) — one collective per step
        g.copy_(torch.where(self.bmask, self.params[0] if self.rank == 0 else torch.zeros_like(g), g))
        comm.all_reduce_flat(self.gsum, group=self.pg)
        p0 = self.params[0:1]
        p0.copy_(torch.where(self.bmask, self.gsum, p0))
        self.gsum.masked_fill_(self.bmask.view(1, -1), 0.0)
        self.t += 1
        if self.opt_name == "sgd":
            if self.wd:
                self.gsum.addcmul_(self.wmask.view(1, -1), p0, value=self.wd)     # no decay on BN statistics
            ops.sgd_step(p0, self.gsum, self.lr, momentum=self.momentum, mom_buf=self.mom, first_step=self.t == 1)
        else:
            decoupled = self.opt_name == "adamw"
            if self.wd and decoupled:
                p0.sub_(self.wmask.view(1, -1) * p0, alpha=self.lr * self.wd)
            elif self.wd:
                self.gsum.addcmul_(self.wmask.view(1, -1), p0, value=self.wd)
            ops.adam_step(p0, self.gsum, self.m1, self.m2, torch.full((1,), float(self.t), device=self.device),
                          self.lr, amsgrad=self.vmax is not None, max_exp_avg_sq=self.vmax)
        ops.broadcast_rows_(self.params, p0[0].clone() if self.R > 1 else p0[0])
        return loss / R

    def _sync_module(self):
        """Master weights → the torch module (evaluation, state_dict)."""
        if self.native is not None:
            self.model.load_state_dict(self.layout.unflatten(self.params[0]))

    # ------------------------------------------------------------------ epochs
    def train_epoch(self, epoch):
        losses = []
        n = len(self.train_data.x)
        if self.native is not None:
            Q = self.R * self.world
            rows = [shard_indices(n, self.rank * self.R + r, Q, epoch, self.shuffle, self.seed) for r in range(self.R)]
            idx = torch.stack(rows).to(self.device)
            for s in range(0, idx.shape[1], self.bs):
                losses.append(self._native_step(idx[:, s:s + self.bs]))
                self.samples_seen += idx[:, s:s + self.bs].numel() * self.world
        else:
            self.ddp.train()
            for x, y in shard_batches(self.train_data, self.rank, self.world, self.bs, epoch, self.shuffle,
                                      self.seed):
                x, y = x.to(self.device, non_blocking=True), y.to(self.device, non_blocking=True)
                self.opt.zero_grad()
                with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.compute_dtype is not None):
                    loss = self.crit(self.ddp(x), y)
                loss.backward()
                self.ddp.finish_gradient_sync()
                self.opt.step()
                losses.append(loss.detach())
                self.samples_seen += len(y) * self.world
        return torch.stack(losses).mean() if losses else torch.zeros((), device=self.device)

    @torch.no_grad()
    def evaluate(self):
        """Exact global test accuracy / loss: rank r evaluates samples r, r + W, … (no padding), counts are
        all-reduced."""
        if self.test_data is None:
            return {}
        self._sync_module()
        self.model.eval()
        stats = torch.zeros(3, dtype=torch.float64, device=self.device)  # correct, loss_sum, n
        x_all, y_all = self.test_data.x, self.test_data.y
        mine = torch.arange(self.rank, len(x_all), self.world)
        for s in range(0, len(mine), 512):
            sel = mine[s:s + 512]
            x, y = x_all[sel].to(self.device), y_all[sel].to(self.device)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.compute_dtype is not None):
                out = self.model(x).float()
            stats[0] += (out.argmax(1) == y).sum()
            stats[1] += nn.functional.cross_entropy(out, y, reduction="sum")
            stats[2] += y.numel()
        comm.all_reduce_flat(stats, group=self.pg)
        self.model.train()
        n = max(1.0, float(stats[2]))
        return {"test_acc": float(stats[0]) / n, "test_loss": float(stats[1]) / n}

    def state_dict(self):
        self._sync_module()
        return self.model.state_dict()

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

    def close(self):
        if self.native is not None:
            self.native.close()
