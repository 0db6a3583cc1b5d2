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

* native (GPU): ``replicas_per_gpu`` = R data-parallel replicas of the model are R client slots of the FL simulator's
  client-batched engine (``ClientBatchEngine``): the native HIP ResNet step for CIFAR ResNets, the client-batched
  transformer kernels for DistilBERT / ViT (auto picks them at bf16; fp32 transformers go to torch unless
  ``cheetah_exec: native``). Per-replica BatchNorm, like per-rank BN under DDP. Gradients leave the backward in
  buckets (``GradBuckets``): the kernels report which gradient-arena columns they finished
  (``transformer_ops.grad_ready_listener``; torch-accumulated leaves through post-accumulate hooks), and each complete
  run of columns is averaged over the local replicas (``weighted_sum`` kernel) and all-reduced asynchronously while
  the rest of the backward is still being issued; the fused optimizer then updates master row 0 bucket by bucket as
  the all-reduces land, and one broadcast launch copies it to the R rows. BatchNorm running statistics follow
  replica 0 of rank 0 (torch DDP's ``broadcast_buffers``): rank 0's replica-0 statistics are only ever updated by its
  own batches, so they are broadcast once when the module is synchronised (evaluation, ``state_dict``), never per
  step.
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
from ..ops import transformer_ops as T
from ..parallel import comm
from .ddp import FlatDDP, FlatOptimizer


class GradBuckets:
    """Bucketed, backward-overlapped gradient reduction of an [R, P] replica gradient arena: columns complete as the
    backward's Functions report them (``ready``); every maximal run of complete columns at the top of the pending
    range that reaches ``bucket_mb`` is averaged over the R local replicas into ``gsum`` (one ``weighted_sum``
    launch on the compute stream, after the writes) and all-reduced asynchronously (RCCL's stream waits on the
    compute stream's event, so the collective overlaps the rest of the backward). Backward writes gradients from
    the last layer to the first, i.e. from high to low arena offsets, so the runs form as the backward proceeds.
    ``finish`` issues the rest and yields each bucket's (lo, hi) as its all-reduce completes."""

    def __init__(self, layout, grads, rep_w, gsum, group, bucket_mb):
        self.grads, self.rep_w, self.gsum, self.group = grads, rep_w, gsum, group
        self.P = layout.size
        self.B = max(1024, int(bucket_mb * (1 << 20) / 4))
        self.ld = grads.stride(0)
        self.es = grads.element_size()
        ts = sorted((s.offset, s.numel) for s in layout.slots if s.trainable)
        self.lo_of = [o for o, _ in ts]                       # trainable slot starts, ascending
        self.end_of = {o: o + n for o, n in ts}
        self.launched_during_backward = 0

    def begin(self):
        self.done = set()
        self.hi = self.P                # columns [hi, P) are launched
        self.k = len(self.lo_of) - 1    # highest trainable slot not yet launched
        self.works = []

    def _launch(self, lo, hi):
        if hi <= lo:
            return
        ops.weighted_sum(self.grads[:, lo:hi], self.rep_w, out=self.gsum[0, lo:hi])
        self.works.append((lo, hi, comm.all_reduce_flat(self.gsum[0, lo:hi], group=self.group, async_op=True)))

    def ready(self, views):
        base = self.grads.data_ptr()
        for v in views:
            off = ((v.data_ptr() - base) // self.es) % self.ld
            if off in self.end_of:
                self.done.add(off)
        # extend the complete run downward from the launched boundary; launch once it holds a bucket
        lo = self.hi
        k = self.k
        while k >= 0 and self.lo_of[k] in self.done:
            lo = self.lo_of[k]
            k -= 1
        if self.hi - lo >= self.B:
            self._launch(lo, self.hi)
            self.hi, self.k = lo, k
            self.launched_during_backward += 1

    def finish(self):
        self._launch(0, self.hi)
        self.hi = 0
        for lo, hi, ws in self.works:
            for w in ws:
                w.wait()
            yield lo, hi


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
        if mode == "native" or (mode == "auto" and self.device.type == "cuda"):
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
        """The client-batched engine of the FL simulator as the replica executor: R replicas are R client slots
        (``ClientBatchEngine``: the native HIP ResNet step, or the client-batched transformer kernels for
        DistilBERT / ViT). Anything else (its executor would be the torch interpreter) keeps ``FlatDDP``."""
        from ..simulation.rccl.engine import ClientBatchEngine
        eng = ClientBatchEngine(self.model, R, self.device, self.args, self.compute_dtype)
        if eng.executor == "transformer" and self.compute_dtype is None and not required:
            # fp32 transformers: the client-batched fp32 GEMMs trail hipBLASLt's fp32 GEMMs on one GPU (ViT-B/16 595
            # vs 804, DistilBERT 2121 vs 2717 samples/s, profiles/r6_bench_lines.txt); bf16 is the native win
            # (2266 vs 1722, 7650 vs 6199). cheetah_exec: native forces the native executor anyway.
            eng.close()
            logging.info("cheetah: torch executor for an fp32 transformer (cheetah_exec: native overrides)")
            return
        if eng.executor not in ("native", "transformer"):
            eng.close()
            if required:
                from ..parallel.native_resnet import UnsupportedNative
                raise UnsupportedNative(f"no native replica executor for this model ({eng.executor})")
            logging.info("cheetah: torch executor (engine would run %s)", eng.executor)
            return
        self.engine, self.native, self.layout, self.R = eng, eng.native_step or eng.tf, eng.layout, R
        dev = self.device
        layout = self.layout
        self.params, self.grads = eng.params, eng.grads
        flat = layout.flatten(self.model.state_dict(), device=dev)
        comm.broadcast_flat(flat, 0, self.pg)               # every rank starts from rank 0's weights
        eng.load_global(flat)
        P = layout.size
        self.gsum = torch.zeros(1, P, dtype=torch.float32, device=dev)
        self.tmask = layout.trainable_mask(dev).to(torch.bool)
        self.wmask = self.tmask.to(torch.float32) if self.wd else None
        self.mom = torch.zeros(1, P, device=dev) if (self.opt_name == "sgd" and self.momentum) else None
        if self.opt_name != "sgd":
            self.m1 = torch.zeros(1, P, device=dev)
            self.m2 = torch.zeros(1, P, device=dev)
            self.vmax = torch.zeros(1, P, device=dev) if self.opt_name == "adam" else None
        self.t = 0
        self.rep_w = torch.full((R,), 1.0 / (R * self.world), dtype=torch.float32, device=dev)
        self.active = torch.ones(R, dtype=torch.float32, device=dev)
        self.x_dev = self.train_data.x.to(dev, non_blocking=True)
        self.y_dev = self.train_data.y.to(dev, non_blocking=True)
        self.buckets = GradBuckets(layout, self.grads, self.rep_w, self.gsum, self.pg,
                                   float(getattr(self.args, "ddp_bucket_mb", 64.0) or 64.0))
        # CPU / torch-accumulated gradients report completion through post-accumulate hooks; the native kernels
        # report it themselves (transformer_ops grad_ready_listener)
        self._hooks = [v.register_post_accumulate_grad_hook(lambda t: self.buckets.ready([t.grad]))
                       for v in eng.views.values() if v.requires_grad]

    def _native_step(self, idx):
        """idx [R, b] sample indices (one row per local replica). Backward runs under the bucketer: each bucket of
        gradient columns whose writes are all enqueued is averaged over the local replicas (``weighted_sum``) and
        its all-reduce starts on RCCL's stream while the rest of the backward still runs; the optimizer then
        updates each bucket as its all-reduce lands."""
        R, b = idx.shape
        x = self.x_dev[idx.reshape(-1)].view(R, b, *self.x_dev.shape[1:])
        if x.is_floating_point():
            x = x.float()
        y = self.y_dev[idx.reshape(-1)].view(R, b).long()
        mask = self._masks.get(b) if hasattr(self, "_masks") else None
        if mask is None:
            self._masks = getattr(self, "_masks", {})
            mask = self._masks[b] = torch.ones(R, b, dtype=torch.bool, device=self.device)
        eng = self.engine
        self.buckets.begin()
        with T.grad_ready_listener(self.buckets.ready):
            loss = eng._step_loss(x, y, mask, [b] * R, self.active, None, self.device.type == "cuda")
        self.t += 1
        for lo, hi in self.buckets.finish():
            self._opt_slice(lo, hi)
        ops.broadcast_rows_(self.params, self.params[0].clone() if self.R > 1 else self.params[0])
        eng._shadow_stale = True
        return loss / R

    def _opt_slice(self, lo, hi):
        """Fused optimizer on master row 0, columns [lo, hi) (BatchNorm statistics / counters have zero gradients
        and no decay: they are left as replica 0 computed them)."""
        p0, g = self.params[0:1, lo:hi], self.gsum[:, lo:hi]
        wm = self.wmask[lo:hi].view(1, -1) if self.wd else None
        if self.opt_name == "sgd":
            if self.wd:
                g.addcmul_(wm, p0, value=self.wd)
            ops.sgd_step(p0, g, self.lr, momentum=self.momentum,
                         mom_buf=self.mom[:, lo:hi] if self.mom is not None else None, first_step=self.t == 1)
        else:
            decoupled = self.opt_name == "adamw"
            if self.wd and decoupled:
                p0.sub_(wm * p0, alpha=self.lr * self.wd)
            elif self.wd:
                g.addcmul_(wm, p0, value=self.wd)
            ops.adam_step(p0, g, self.m1[:, lo:hi], self.m2[:, lo:hi],
                          torch.full((1,), float(self.t), device=self.device), self.lr, amsgrad=self.vmax is not None,
                          max_exp_avg_sq=self.vmax[:, lo:hi] if self.vmax is not None else None)

    def set_data(self, train):
        """Swap the training data (a ``ClientData``-like object; the silo adapter's next data index)."""
        self.train_data = train
        if self.native is not None:
            self.x_dev = train.x.to(self.device, non_blocking=True)
            self.y_dev = train.y.to(self.device, non_blocking=True)

    def load_state(self, state_dict, broadcast: bool = True):
        """New starting weights on every replica (a new FL round) with a fresh optimizer state. ``broadcast``:
        take rank 0's (False when the caller's ranks already hold the same state, e.g. after the silo's own sync)."""
        if self.native is None:
            self.model.load_state_dict(state_dict)
            return
        flat = self.layout.flatten(state_dict, device=self.device)
        if broadcast:
            comm.broadcast_flat(flat, 0, self.pg)
        self.engine.load_global(flat)
        self.t = 0
        for buf in (self.mom, getattr(self, "m1", None), getattr(self, "m2", None), getattr(self, "vmax", None)):
            if buf is not None:
                buf.zero_()

    def _sync_module(self):
        """Master weights → the torch module (evaluation, state_dict). Trainable weights are identical on every
        rank; BatchNorm running statistics follow replica 0 of rank 0 (torch DDP's broadcast_buffers: rank 0's
        replica-0 statistics are only ever updated by its own batches, so broadcasting them once here equals
        broadcasting them before every forward)."""
        if self.native is not None:
            flat = self.params[0].clone()
            if comm.is_dist():
                # only the buffer columns differ between ranks (none for a transformer: no collective at all)
                if getattr(self, "_bufcols", None) is None:
                    self._bufcols = torch.nonzero(~self.tmask).view(-1)
                if self._bufcols.numel():
                    b = flat.index_select(0, self._bufcols)
                    comm.broadcast_flat(b, 0, self.pg)
                    flat.index_copy_(0, self._bufcols, b)
            self.model.load_state_dict(self.layout.unflatten(flat))

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
            for h in self._hooks:
                h.remove()
            self.engine.close()
