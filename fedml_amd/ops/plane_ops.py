"""Client-batched depthwise convolution and BatchNorm(+ReLU) on the batched interpreter's client-stacked NCHW
activations ``[B, C·Ch, H, W]`` (``csrc/plane_kernels.hip``) — the MobileNet family's depthwise-separable
blocks (reference ``model/cv/mobilenet.py:58-150``, ``mobilenet_v3.py:148-316``) without MIOpen's grouped
convolution or batch-norm kernels.

* :func:`depthwise_conv2d` — per-client ``[C, Ch, 1, k, k]`` filters (arena views), k ∈ {3, 5, 7}, stride 1/2,
  pad k//2; backward gives dx and the per-client weight gradient (deterministic per-channel reductions).
* :func:`plane_batch_norm` — training-mode BN with per-client affine ``[C, Ch]`` (arena views), optionally
  fused with the following ReLU (the mask is recomputed from the input in backward, no extra tensor);
  returns the batch mean / biased variance for the caller's running-statistics update.

Storage precision = the activation dtype (fp32, the reference's, or bf16); statistics fp32."""
import ctypes as _c

import torch

from .fl_ops import _check, _f, _fn, _i64, _p, _stream


def _bf(t):
    return int(t.dtype == torch.bfloat16)


def _owns_grad(p) -> bool:
    """``p`` is a leaf whose ``.grad`` is a pre-assigned fp32 view with contiguous per-client rows (the batched
    engine's gradient arena): the kernels accumulate into it directly and autograd gets no gradient to add."""
    g = getattr(p, "grad", None) if p is not None else None
    return (p is not None and p.is_leaf and p.requires_grad and g is not None and g.dtype == torch.float32
            and g.shape == p.shape and g[0].is_contiguous())


class _PbnExt(_c.Structure):
    _fields_ = [("rm", _c.c_void_p), ("rv", _c.c_void_p), ("nbt", _c.c_void_p), ("rcs", _c.c_int64),
                ("momentum", _c.c_float), ("active", _c.c_void_p), ("dg", _c.c_void_p), ("db", _c.c_void_p),
                ("dcs", _c.c_int64)]


def depthwise_module(m) -> bool:
    """The layer shape alone: a depthwise convolution the plane kernels take (no bias)."""
    k = m.kernel_size
    return (m.groups == m.in_channels == m.out_channels and m.groups > 1 and k[0] == k[1] and k[0] in (3, 5, 7)
            and m.stride[0] == m.stride[1] and m.stride[0] in (1, 2) and isinstance(m.padding, tuple)
            and m.padding == (k[0] // 2, k[0] // 2) and m.dilation == (1, 1) and m.padding_mode == "zeros"
            and m.bias is None)


def supported_dw(m, x, w) -> bool:
    """nn.Conv2d ``m`` is a depthwise layer the kernels take, on client-stacked ``x`` with weights ``w``."""
    k = m.kernel_size
    return (x.is_cuda and x.dim() == 4 and x.dtype in (torch.float32, torch.bfloat16) and x.is_contiguous()
            and m.groups == m.in_channels == m.out_channels and k[0] == k[1] and k[0] in (3, 5, 7)
            and m.stride[0] == m.stride[1] and m.stride[0] in (1, 2) and isinstance(m.padding, tuple)
            and m.padding == (k[0] // 2, k[0] // 2) and m.dilation == (1, 1) and m.padding_mode == "zeros"
            and w.dtype == torch.float32 and w[0].is_contiguous())


class _DWConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, C, stride):
        B, CC, H, W = x.shape
        Ch, K = w.shape[1], w.shape[-1]
        Ho, Wo = (H + 2 * (K // 2) - K) // stride + 1, (W + 2 * (K // 2) - K) // stride + 1
        y = torch.empty(B, CC, Ho, Wo, dtype=x.dtype, device=x.device)
        rc = _fn("fa_dwconv")(_c.c_int(0), _c.c_int(_bf(x)), _p(x), None, _p(w), _i64(w.stride(0)), _p(y),
                              _c.c_int(B), _c.c_int(CC), _c.c_int(Ch), _c.c_int(H), _c.c_int(W), _c.c_int(Ho),
                              _c.c_int(Wo), _c.c_int(K), _c.c_int(stride), _stream(x))
        _check(rc, "fa_dwconv fwd")
        ctx.save_for_backward(x, w)
        ctx.cfg = (C, stride, Ho, Wo)
        ctx.w_ref = w            # the leaf itself (its pre-assigned .grad view), not the saved-tensor copy
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        C, stride, Ho, Wo = ctx.cfg
        B, CC, H, W = x.shape
        Ch, K = w.shape[1], w.shape[-1]
        gy = gy.to(x.dtype).contiguous()
        dx = dw = None
        args = (_c.c_int(B), _c.c_int(CC), _c.c_int(Ch), _c.c_int(H), _c.c_int(W), _c.c_int(Ho), _c.c_int(Wo),
                _c.c_int(K), _c.c_int(stride), _stream(x))
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            rc = _fn("fa_dwconv")(_c.c_int(1), _c.c_int(_bf(x)), _p(gy), None, _p(w), _i64(w.stride(0)), _p(dx), *args)
            _check(rc, "fa_dwconv bwd_data")
        if ctx.needs_input_grad[1]:
            if _owns_grad(ctx.w_ref):   # the engine's gradient-arena view: accumulate in the kernel
                g = ctx.w_ref.grad
                rc = _fn("fa_dwconv")(_c.c_int(2), _c.c_int(_bf(x)), _p(gy), _p(x), None, _i64(g.stride(0)), _p(g),
                                      *args)
            else:
                dw = torch.empty(C, Ch, 1, K, K, dtype=torch.float32, device=x.device)
                rc = _fn("fa_dwconv")(_c.c_int(2), _c.c_int(_bf(x)), _p(gy), _p(x), None, _i64(0), _p(dw), *args)
            _check(rc, "fa_dwconv wgrad")
        return dx, dw, None, None


def depthwise_conv2d(x, w, C, stride):
    """x [B, C·Ch, H, W]; w [C, Ch, 1, k, k] fp32 (client-stacked arena view) → [B, C·Ch, Ho, Wo]."""
    return _DWConv.apply(x.contiguous(), w, int(C), int(stride))


class _PlaneBN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, C, eps, relu, stats_out, running):
        B, CC, H, W = x.shape
        Ch = CC // C
        mean = torch.empty(CC, dtype=torch.float32, device=x.device)
        var = torch.empty(CC, dtype=torch.float32, device=x.device)
        pcs = weight.stride(0) if weight is not None else 0
        common = (_p(weight), _p(bias), _i64(pcs), _p(mean), _p(var), _f(eps), _c.c_int(int(relu)))
        ext = None
        if running is not None:   # (running_mean, running_var, num_batches_tracked | None, momentum, active | None)
            rm, rv, nbt, mom, active = running
            ext = _PbnExt(rm.data_ptr(), rv.data_ptr(), nbt.data_ptr() if nbt is not None else None, rm.stride(0),
                          float(mom), active.data_ptr() if active is not None else None, None, None, 0)
        rc = _fn("fa_plane_bn")(_c.c_int(0), _c.c_int(_bf(x)), _p(x), None, None, *common, None, _c.c_int(B),
                                _c.c_int(CC), _c.c_int(Ch), _c.c_int(H * W), _c.byref(ext) if ext is not None else None,
                                _stream(x))
        _check(rc, "fa_plane_bn stats")
        dims = (_c.c_int(B), _c.c_int(CC), _c.c_int(Ch), _c.c_int(H * W), None, _stream(x))
        y = torch.empty_like(x)
        rc = _fn("fa_plane_bn")(_c.c_int(1), _c.c_int(_bf(x)), _p(x), None, _p(y), *common, None, *dims)
        _check(rc, "fa_plane_bn apply")
        stats_out.append((mean.view(C, Ch), var.view(C, Ch), float(B * H * W)))
        ctx.save_for_backward(x, weight, bias, mean, var)
        ctx.cfg = (C, eps, relu)
        ctx.wb_ref = (weight, bias)   # the leaves themselves (their pre-assigned .grad views)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, weight, bias, mean, var = ctx.saved_tensors
        C, eps, relu = ctx.cfg
        B, CC, H, W = x.shape
        Ch = CC // C
        gy = gy.to(x.dtype).contiguous()
        pcs = weight.stride(0) if weight is not None else 0
        red = torch.empty(CC, 2, dtype=torch.float32, device=x.device)
        common = (_p(weight), _p(bias), _i64(pcs), _p(mean), _p(var), _f(eps), _c.c_int(int(relu)))
        # dγ / dβ straight into the engine's gradient-arena rows when it owns them (one writer per element)
        wl, bl = ctx.wb_ref
        own = (wl is not None and bl is not None and _owns_grad(wl) and _owns_grad(bl)
               and wl.grad.stride(0) == bl.grad.stride(0))
        ext = _PbnExt(None, None, None, 0, 0.0, None, wl.grad.data_ptr(), bl.grad.data_ptr(),
                      wl.grad.stride(0)) if own else None
        rc = _fn("fa_plane_bn")(_c.c_int(2), _c.c_int(_bf(x)), _p(x), _p(gy), None, *common, _p(red), _c.c_int(B),
                                _c.c_int(CC), _c.c_int(Ch), _c.c_int(H * W), _c.byref(ext) if own else None,
                                _stream(x))
        _check(rc, "fa_plane_bn bwd_reduce")
        dims = (_c.c_int(B), _c.c_int(CC), _c.c_int(Ch), _c.c_int(H * W), None, _stream(x))
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            rc = _fn("fa_plane_bn")(_c.c_int(3), _c.c_int(_bf(x)), _p(x), _p(gy), _p(dx), *common, _p(red), *dims)
            _check(rc, "fa_plane_bn dx")
        if own:
            return dx, None, None, None, None, None, None, None
        rs = torch.rsqrt(var + eps)
        dg = (red[:, 1] * rs).view(C, Ch) if weight is not None else None
        db = red[:, 0].view(C, Ch) if bias is not None else None
        return dx, dg, db, None, None, None, None, None


def plane_batch_norm(x, weight, bias, C, eps, relu=False, running=None):
    """Training BN(+ReLU) of client-stacked x [B, C·Ch, H, W] with per-client affine [C, Ch] (or None).
    Returns (y, (mean [C, Ch], biased var [C, Ch], n)) — the batch statistics. ``running`` = (running_mean,
    running_var [C, Ch] fp32 views sharing one client stride, num_batches_tracked [C] view or None, momentum,
    active [C] or None): the statistics kernel also updates them (torch's training-mode rule: momentum, unbiased
    variance; active clients only) — no separate update pass."""
    stats = []
    if running is not None:
        rm, rv, nbt = running[:3]
        assert rm.dtype == rv.dtype == torch.float32 and rm.stride() == rv.stride() and rm[0].is_contiguous()
        assert nbt is None or (nbt.dtype == torch.float32 and nbt.stride(0) == rm.stride(0))
    y = _PlaneBN.apply(x.contiguous(), weight, bias, int(C), float(eps), bool(relu), stats, running)
    return y, stats[0]


def plane_supported(x, weight, C) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype in (torch.float32, torch.bfloat16) and x.shape[1] % C == 0
            and (weight is None or (weight.dtype == torch.float32 and weight[0].is_contiguous())))
