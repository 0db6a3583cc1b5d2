"""GroupNorm over the HIP kernels of ``csrc/gn_kernels.hip``.

The reference builds GroupNorm out of ``F.batch_norm`` on a reshaped ``[1, N·G, ...]`` copy
(``model/cv/group_normalization.py:7-93``); here one kernel normalises a group row per workgroup
(fp32 statistics, bf16 or fp32 activations, optional fused ReLU) and one kernel computes dx together
with dγ/dβ. ``clients > 1`` runs the client-stacked layout of the virtual-client engine: ``x`` is
``[N, clients·ch, H, W]`` and weight/bias are ``[clients, ch]`` (strided fp32 arena views are read
in place). CPU tensors run the PyTorch reference (the oracle of the GPU tests).
"""
import ctypes as _c

import torch
import torch.nn as nn
import torch.nn.functional as F

from .fl_ops import _check, _f, _fn, _i64, _p, _stream, use_native


def _fp32_rows(t):
    if t is None:
        return None
    return t if (t.dtype == torch.float32 and t.stride(-1) == 1) else t.float().contiguous()


def _gn_ref(x, groups, weight, bias, eps, relu, clients):
    Ct = x.shape[1]
    y = F.group_norm(x.float(), groups * clients, None, None, eps)
    shape = (1, Ct) + (1,) * (x.dim() - 2)
    if weight is not None:
        y = y * weight.reshape(shape).float()
    if bias is not None:
        y = y + bias.reshape(shape).float()
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype)


class _GroupNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, R, clients, eps, relu):
        N, Ct = x.shape[:2]
        HW = x[0, 0].numel()
        w2, b2 = _fp32_rows(weight), _fp32_rows(bias)
        y = torch.empty_like(x)
        mean = torch.empty(N * R, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        dt = 1 if x.dtype == torch.bfloat16 else 0
        rc = _fn("fa_gn_fwd")(_p(x), _p(y), _p(w2), _i64(w2.stride(0) if w2 is not None else 0), _p(b2),
                              _i64(b2.stride(0) if b2 is not None else 0), _c.c_int(Ct // clients), _p(mean),
                              _p(rstd), _i64(N * R), _c.c_int(R), _c.c_int(Ct // R), _c.c_int(HW), _f(eps),
                              _c.c_int(int(relu)), _c.c_int(dt), _stream(x))
        _check(rc, "fa_gn_fwd")
        ctx.save_for_backward(x, y if relu else None, mean, rstd)
        ctx.cfg = (R, clients, relu, w2, weight is not None, bias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mean, rstd = ctx.saved_tensors
        R, clients, relu, w2, has_w, has_b = ctx.cfg
        N, Ct = x.shape[:2]
        HW = x[0, 0].numel()
        dy = dy.contiguous()
        if relu:
            dy = dy * (y > 0).to(dy.dtype)
        dx = torch.empty_like(x)
        dw = torch.zeros(Ct, dtype=torch.float32, device=x.device) if has_w and ctx.needs_input_grad[1] else None
        db = torch.zeros(Ct, dtype=torch.float32, device=x.device) if has_b and ctx.needs_input_grad[2] else None
        dt = 1 if x.dtype == torch.bfloat16 else 0
        rc = _fn("fa_gn_bwd")(_p(dy), _p(x), _p(w2), _i64(w2.stride(0) if w2 is not None else 0),
                              _c.c_int(Ct // clients), _p(mean), _p(rstd), _p(dx), _p(dw), _p(db), _i64(N * R),
                              _c.c_int(R), _c.c_int(Ct // R), _c.c_int(HW), _c.c_int(dt), _stream(x))
        _check(rc, "fa_gn_bwd")
        gw = dw.view(clients, -1) if dw is not None else None
        gb = db.view(clients, -1) if db is not None else None
        return dx, gw, gb, None, None, None, None


def group_norm(x: torch.Tensor, num_groups: int, weight=None, bias=None, eps: float = 1e-5, relu: bool = False,
               clients: int = 1) -> torch.Tensor:
    """GroupNorm with ``num_groups`` groups per client (+ fused ReLU) of an N·C·… tensor ``x``;
    weight/bias are ``[ch]`` (one model) or ``[clients, ch]`` (client-stacked)."""
    assert x.shape[1] % (num_groups * clients) == 0
    if use_native(x) and x.dtype in (torch.float32, torch.bfloat16):
        w = weight.reshape(clients, -1) if weight is not None else None
        b = bias.reshape(clients, -1) if bias is not None else None
        return _GroupNorm.apply(x.contiguous(), w, b, num_groups * clients, clients, float(eps), bool(relu))
    return _gn_ref(x, num_groups, weight, bias, eps, relu, clients)


class FusedGroupNorm(nn.GroupNorm):
    """``nn.GroupNorm`` whose forward runs the HIP kernels on GPU tensors (same parameters and
    state_dict keys; bf16 activations stay bf16 instead of autocast's fp32 upcast)."""

    def forward(self, x):
        return group_norm(x, self.num_groups, self.weight, self.bias, self.eps)


def fuse_group_norm(model: nn.Module) -> int:
    """Switch every ``nn.GroupNorm`` of ``model`` to :class:`FusedGroupNorm` in place."""
    n = 0
    for m in model.modules():
        if type(m) is nn.GroupNorm:
            m.__class__ = FusedGroupNorm
            n += 1
    return n
