"""Cross-GPU synchronised BatchNorm (reference: ``model/cv/batchnorm_utils.py`` — SynchronizedBatchNorm
1d/2d/3d for single-process ``DataParallel`` with a thread master/slave pipe and replication callbacks).

MI355X-native design: one process per GPU, so the batch statistics are reduced with ONE
``torch.distributed`` all-reduce per layer and direction (RCCL over xGMI; gloo on CPU) of a packed
[Σx ‖ Σx² ‖ n] (forward) or [Σdy ‖ Σdy·x̂] (backward) vector — 2C+1 floats, latency-bound, so one
message. Without an initialised process group it is plain BatchNorm. The thread pipes / replication
callbacks of the reference have no counterpart (there are no replicas inside a process)."""
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from ...parallel import comm


class _SyncBNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps, group):
        C = x.shape[1]
        dims = [0] + list(range(2, x.dim()))
        xf = x.float()
        n_local = float(x.numel() // C)
        buf = torch.cat([xf.sum(dims), (xf * xf).sum(dims), torch.tensor([n_local], device=x.device)])
        if comm.is_dist():
            dist.all_reduce(buf, group=group)
        n = buf[2 * C]
        mean = buf[:C] / n
        var = (buf[C:2 * C] / n - mean * mean).clamp_min(0.0)
        invstd = torch.rsqrt(var + eps)
        shape = [1, C] + [1] * (x.dim() - 2)
        xhat = (xf - mean.view(shape)) * invstd.view(shape)
        y = xhat * weight.float().view(shape) + bias.float().view(shape) if weight is not None else xhat
        ctx.save_for_backward(xhat, invstd, weight)
        ctx.group, ctx.n, ctx.dims = group, n, dims
        return y.to(x.dtype), mean, var * n / (n - 1).clamp_min(1.0)

    @staticmethod
    def backward(ctx, dy, _dm, _dv):
        xhat, invstd, weight = ctx.saved_tensors
        C = xhat.shape[1]
        shape = [1, C] + [1] * (xhat.dim() - 2)
        dyf = dy.float()
        local = torch.cat([dyf.sum(ctx.dims), (dyf * xhat).sum(ctx.dims)])
        dbias, dweight = local[:C].clone(), local[C:].clone()       # parameter grads: this rank's share
        if comm.is_dist():
            dist.all_reduce(local, group=ctx.group)
        mdy, mdyx = local[:C] / ctx.n, local[C:] / ctx.n
        g = weight.float().view(shape) if weight is not None else 1.0
        dx = g * invstd.view(shape) * (dyf - mdy.view(shape) - xhat * mdyx.view(shape))
        return dx.to(dy.dtype), (dweight if weight is not None else None), (dbias if weight is not None else None), \
            None, None


class _SynchronizedBatchNorm(nn.modules.batchnorm._BatchNorm):
    """BatchNorm whose training statistics span every rank of ``process_group`` (default: WORLD)."""

    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, track_running_stats=True,
                 process_group=None):
        super().__init__(num_features, eps, momentum, affine, track_running_stats)
        self.process_group = process_group

    def forward(self, x):
        self._check_input_dim(x)
        if not self.training:
            return F.batch_norm(x, self.running_mean, self.running_var, self.weight, self.bias, False, 0.0, self.eps)
        y, mean, var_unbiased = _SyncBNFn.apply(x, self.weight, self.bias, self.eps, self.process_group)
        if self.track_running_stats:
            with torch.no_grad():
                self.num_batches_tracked.add_(1)
                m = self.momentum if self.momentum is not None else 1.0 / float(self.num_batches_tracked)
                self.running_mean.mul_(1 - m).add_(mean.to(self.running_mean.dtype), alpha=m)
                self.running_var.mul_(1 - m).add_(var_unbiased.to(self.running_var.dtype), alpha=m)
        return y


class SynchronizedBatchNorm1d(_SynchronizedBatchNorm):
    def _check_input_dim(self, x):
        if x.dim() not in (2, 3):
            raise ValueError(f"expected 2D or 3D input (got {x.dim()}D)")


class SynchronizedBatchNorm2d(_SynchronizedBatchNorm):
    def _check_input_dim(self, x):
        if x.dim() != 4:
            raise ValueError(f"expected 4D input (got {x.dim()}D)")


class SynchronizedBatchNorm3d(_SynchronizedBatchNorm):
    def _check_input_dim(self, x):
        if x.dim() != 5:
            raise ValueError(f"expected 5D input (got {x.dim()}D)")


def convert_sync_batchnorm(module: nn.Module, process_group=None) -> nn.Module:
    """Replace every BatchNorm{1,2,3}d (parameters and running statistics kept) by its synchronised
    twin — the process-per-GPU replacement for ``DataParallelWithCallback`` + ``patch_replication_callback``."""
    kinds = {nn.BatchNorm1d: SynchronizedBatchNorm1d, nn.BatchNorm2d: SynchronizedBatchNorm2d,
             nn.BatchNorm3d: SynchronizedBatchNorm3d}
    out = module
    t = kinds.get(type(module))
    if t is not None:
        out = t(module.num_features, module.eps, module.momentum, module.affine, module.track_running_stats,
                process_group)
        if module.affine:
            with torch.no_grad():
                out.weight.copy_(module.weight)
                out.bias.copy_(module.bias)
        if module.track_running_stats:
            out.running_mean.copy_(module.running_mean)
            out.running_var.copy_(module.running_var)
            out.num_batches_tracked.copy_(module.num_batches_tracked)
        out.train(module.training)
    for name, child in module.named_children():
        out.add_module(name, convert_sync_batchnorm(child, process_group))
    return out
