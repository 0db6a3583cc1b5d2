"""Channels-last training BatchNorm (+ residual add + ReLU) over ``csrc/bnc_kernels.hip``.

The reference runs ``nn.BatchNorm2d`` then ``nn.ReLU`` (and ``out += identity``) as separate cuDNN / ATen
kernels after every convolution of its CIFAR ResNets (``model/cv/resnet.py:38-120``). On the per-client
(wide-CNN) path of the virtual-client engine that is MIOpen's six batch-norm kernels per layer plus the
elementwise add / ReLU kernels; :func:`batch_norm_act` does the whole ``act(bn(x) [+ residual])`` in two
forward and two backward launches on NHWC bf16 activations (fp32 statistics and parameters; running
statistics updated in place, so arena aliases of them stay live).

Anything the kernels do not cover (CPU, fp32 activations, NCHW layout, eval mode, cumulative-average
momentum, fx tracing, functorch transforms) runs the plain module path — also the oracle of the GPU test.
``FEDML_AMD_BNC=0`` forces the module path for A/B measurements.
"""
import ctypes as _c
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .fl_ops import _check, _f, _fn, _i64, _p, _stream

_ENABLED = os.environ.get("FEDML_AMD_BNC", "1") != "0"


def _shape_ok(C):
    return 8 <= C <= 2048 and C % 8 == 0 and 256 % (C // 8) == 0


def _fast_ok(bn, x, residual):
    if isinstance(x, torch.fx.Proxy) or not _ENABLED:
        return False
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and bn.training):
        return False
    if torch._C._functorch.is_functorch_wrapped_tensor(x):
        return False
    if type(bn) is not nn.BatchNorm2d or not _shape_ok(x.shape[1]):
        return False
    if bn.track_running_stats and (bn.momentum is None or bn.running_mean is None):
        return False
    for t in (bn.weight, bn.bias, bn.running_mean if bn.track_running_stats else None,
              bn.running_var if bn.track_running_stats else None):
        if t is not None and (t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda):
            return False
    if residual is not None and (residual.shape != x.shape or residual.dtype != x.dtype or
                                 residual.data_ptr() % 16):
        return False
    return x.data_ptr() % 16 == 0     # 16-B vector accesses


_CL = torch.channels_last


class _BNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, rmean, rvar, momentum, eps, relu):
        x = x.contiguous(memory_format=_CL)
        if residual is not None:
            residual = residual.contiguous(memory_format=_CL)
        C = x.shape[1]
        M = x.numel() // C
        acc = torch.zeros(2 * C, dtype=torch.float32, device=x.device)   # fwd Σ(x−K), Σ(x−K)²
        save = torch.empty(2 * C, dtype=torch.float32, device=x.device)  # mean, invstd
        y = torch.empty_like(x, memory_format=_CL)
        rc = _fn("fa_bnc_fwd")(_p(x), _p(residual), _p(y), _i64(M), _c.c_int(C), _p(acc), _p(weight), _p(bias),
                               _f(eps), _f(momentum), _p(rmean), _p(rvar), _p(save), _c.c_int(int(relu)),
                               _stream(x))
        _check(rc, "fa_bnc_fwd")
        ctx.save_for_backward(x, y if relu else None, weight, save)
        ctx.relu, ctx.has_res, ctx.M, ctx.has_b = relu, residual is not None, M, bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, weight, save = ctx.saved_tensors
        dy = dy.contiguous(memory_format=_CL)
        if dy.data_ptr() % 16:
            dy = dy.clone(memory_format=_CL)
        C, M = x.shape[1], ctx.M
        # the backward sums are accumulated atomically: a fresh zeroed buffer on EVERY backward (a second
        # backward through a retained graph must not add onto the first one's sums, and a saved tensor must
        # not be modified in place)
        bacc = torch.zeros(2 * C, dtype=torch.float32, device=x.device)
        dx = torch.empty_like(x, memory_format=_CL)
        dres = torch.empty_like(x, memory_format=_CL) if (ctx.has_res and ctx.relu) else None
        dw = torch.empty(C, dtype=torch.float32, device=x.device) if weight is not None else None
        db = torch.empty(C, dtype=torch.float32, device=x.device) if ctx.has_b else None
        rc = _fn("fa_bnc_bwd")(_p(dy), _p(x), _p(y), _p(dres), _p(dx), _i64(M), _c.c_int(C), _p(save),
                               _p(bacc), _p(weight), _p(dw), _p(db), _stream(x))
        _check(rc, "fa_bnc_bwd")
        if ctx.has_res and not ctx.relu:
            dres = dy
        return dx, dw, db, dres, None, None, None, None, None


def batch_norm_act(bn: nn.Module, x: torch.Tensor, residual: torch.Tensor = None, relu: bool = False):
    """``act(bn(x) [+ residual])`` — one fused HIP pass per direction on NHWC bf16 GPU activations,
    the module path otherwise (identical semantics, including ``num_batches_tracked``)."""
    if not _fast_ok(bn, x, residual):
        out = bn(x)
        if residual is not None:
            out = out + residual
        return F.relu(out) if relu else out
    if bn.track_running_stats and bn.num_batches_tracked is not None:
        bn.num_batches_tracked.add_(1)
    track = bn.track_running_stats
    return _BNAct.apply(x, bn.weight, bn.bias, residual, bn.running_mean if track else None,
                        bn.running_var if track else None, float(bn.momentum or 0.0), float(bn.eps), bool(relu))
