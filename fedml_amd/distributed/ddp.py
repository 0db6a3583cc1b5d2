"""Data parallelism over RCCL for one model replicated on every rank ("Cheetah").

``FlatDDP`` is this framework's DistributedDataParallel (the reference wraps torch DDP around
the model inside each silo): trainable parameters are re-homed into ONE flat fp32
arena laid out in *reverse registration order* and every ``p.grad`` is a view of one flat
gradient arena. Backward therefore produces gradients roughly in arena order, so buckets are
contiguous slices: a post-accumulate-grad hook counts ready parameters per bucket and launches
that bucket's asynchronous all-reduce the moment it is complete — communication overlaps the
rest of backward. On MI355X the default bucket (64 MB) is sized for xGMI rings (per-link ~153
GB/s; a 64 MB slice keeps each ring step well above the latency floor), much larger than torch
DDP's 25 MB default tuned for NVLink/NVSwitch. The optimizer then runs as one fused HIP kernel
over the whole arena (``ops.sgd_step`` / ``ops.adam_step``) instead of a per-tensor loop.
"""
import logging
from typing import List, Optional

import torch
import torch.distributed as dist

from .. import ops


class FlatDDP(torch.nn.Module):
    def __init__(self, module: torch.nn.Module, device=None, process_group=None, bucket_mb: float = 64.0,
                 broadcast_buffers: bool = True):
        super().__init__()
        self.module = module
        self.device = torch.device(device) if device is not None else next(module.parameters()).device
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.broadcast_buffers = broadcast_buffers
        params = [p for p in module.parameters() if p.requires_grad]
        self.params = list(reversed(params))  # backward visits the last layers first
        sizes = [p.numel() for p in self.params]
        self.P = int(sum(sizes))
        self.flat = torch.zeros(1, self.P, dtype=torch.float32, device=self.device)
        self.grad = torch.zeros(1, self.P, dtype=torch.float32, device=self.device)
        self.offsets = []
        off = 0
        with torch.no_grad():
            for p, n in zip(self.params, sizes):
                self.flat[0, off:off + n].copy_(p.detach().reshape(-1).float())
                p.data = self.flat[0, off:off + n].view_as(p)
                p.grad = self.grad[0, off:off + n].view_as(p)
                self.offsets.append(off)
                off += n
        # buckets: contiguous arena slices of ≤ bucket_mb
        cap = max(1, int(bucket_mb * (1 << 20)) // 4)
        self.buckets: List[List[int]] = []
        cur, cur_n = [], 0
        for i, n in enumerate(sizes):
            if cur and cur_n + n > cap:
                self.buckets.append(cur)
                cur, cur_n = [], 0
            cur.append(i)
            cur_n += n
        if cur:
            self.buckets.append(cur)
        self.param_bucket = {}
        for b, idxs in enumerate(self.buckets):
            for i in idxs:
                self.param_bucket[i] = b
        self._pending = [len(b) for b in self.buckets]
        self._works = [None] * len(self.buckets)
        self._grad_views = [self.grad[0, o:o + p.numel()].view_as(p) for o, p in zip(self.offsets, self.params)]
        self._callback_queued = False
        self.auto_sync = True  # finish the all-reduce at the end of backward (torch-DDP semantics)
        self._hooks = []
        if self.world > 1:
            for i, p in enumerate(self.params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
            dist.broadcast(self.flat, 0, group=self.pg)
            self._sync_buffers()
        logging.info("FlatDDP: %d params, %.1f MB arena, %d buckets, world %d", len(self.params),
                     self.P * 4 / 2 ** 20, len(self.buckets), self.world)

    # ------------------------------------------------------------------------------------------
    def _bucket_slice(self, b):
        idxs = self.buckets[b]
        lo = self.offsets[idxs[0]]
        hi = self.offsets[idxs[-1]] + self.params[idxs[-1]].numel()
        return self.grad[0, lo:hi]

    def _make_hook(self, i):
        def hook(p):
            gv = self._grad_views[i]
            if p.grad is not gv and p.grad.data_ptr() != gv.data_ptr():
                # an optimizer's zero_grad(set_to_none=True) detached the grad from the arena
                gv.copy_(p.grad)
                p.grad = gv
            if self.auto_sync and not self._callback_queued:
                self._callback_queued = True
                torch.autograd.Variable._execution_engine.queue_callback(self.finish_gradient_sync)
            b = self.param_bucket[i]
            self._pending[b] -= 1
            if self._pending[b] == 0 and self._works[b] is None:
                self._works[b] = dist.all_reduce(self._bucket_slice(b), op=dist.ReduceOp.SUM, group=self.pg,
                                                 async_op=True)
        return hook

    def _sync_buffers(self):
        if not self.broadcast_buffers or self.world <= 1:
            return
        for buf in self.module.buffers():
            if buf.is_floating_point() or buf.dtype in (torch.int64, torch.int32):
                dist.broadcast(buf, 0, group=self.pg)

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    # state dicts are the wrapped model's (no ``module.`` prefix), loads write into the arena
    def state_dict(self, *args, **kwargs):
        return self.module.state_dict(*args, **kwargs)

    def load_state_dict(self, state_dict, strict: bool = True):
        return self.module.load_state_dict(state_dict, strict)

    def zero_grad(self, set_to_none: bool = False):  # grads must stay views of the arena
        self.grad.zero_()

    def finish_gradient_sync(self):
        """Wait for every bucket (launching any that unused parameters left incomplete) and turn
        the SUM into a mean."""
        self._callback_queued = False
        if self.world <= 1 or all(w is None for w in self._works) and all(
                n == len(b) for n, b in zip(self._pending, self.buckets)):
            return  # nothing in flight (e.g. explicit call after the end-of-backward callback ran)
        for b in range(len(self.buckets)):
            if self._works[b] is None:
                self._works[b] = dist.all_reduce(self._bucket_slice(b), op=dist.ReduceOp.SUM, group=self.pg,
                                                 async_op=True)
        for w in self._works:
            w.wait()
        self.grad.mul_(1.0 / self.world)
        self._pending = [len(b) for b in self.buckets]
        self._works = [None] * len(self.buckets)


class FlatOptimizer:
    """Fused SGD(momentum, nesterov, wd) / Adam(W) / AMSGrad over a FlatDDP arena — one kernel
    launch per step on MI355X."""

    def __init__(self, ddp: FlatDDP, name="sgd", lr=0.01, momentum=0.0, weight_decay=0.0, nesterov=False,
                 betas=(0.9, 0.999), eps=1e-8, amsgrad=False):
        self.ddp = ddp
        self.name = name.lower()
        self.lr, self.momentum, self.wd, self.nesterov = lr, momentum, weight_decay, nesterov
        self.betas, self.eps, self.amsgrad = betas, eps, amsgrad
        z = lambda: torch.zeros_like(ddp.flat)  # noqa: E731
        self.mom = z() if (self.name == "sgd" and momentum) else None
        if self.name != "sgd":
            self.m1, self.m2 = z(), z()
            self.vmax = z() if amsgrad else None
        self.t = 0

    def zero_grad(self, set_to_none=False):
        self.ddp.zero_grad()

    @torch.no_grad()
    def step(self):
        self.t += 1
        d = self.ddp
        if self.name == "sgd":
            ops.sgd_step(d.flat, d.grad, self.lr, weight_decay=self.wd, momentum=self.momentum, mom_buf=self.mom,
                         nesterov=self.nesterov, first_step=self.t == 1)
        else:
            step = torch.full((1,), float(self.t), device=d.flat.device)
            ops.adam_step(d.flat, d.grad, self.m1, self.m2, step, self.lr, beta1=self.betas[0], beta2=self.betas[1],
                          eps=self.eps, weight_decay=self.wd, amsgrad=self.amsgrad, max_exp_avg_sq=self.vmax,
                          decoupled=self.name == "adamw")
