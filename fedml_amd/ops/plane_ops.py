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
            dw = torch.empty(C, Ch, 1, K, K, dtype=torch.float32, device=x.device)
            rc = _fn("fa_dwconv")(_c.c_int(2), _c.c_int(_bf(x)), _p(gy), _p(x), None, _i64(0), _p(dw), *args)
            _check(rc, "fa_dwconv wgrad")
        return dx, dw, None, None


def depthwise_conv2d(x, w, C, stride):
    """x [B, C·Ch, H, W]; w [C, Ch, 1, k, k] fp32 (client-stacked arena view) → [B, C·Ch, Ho, Wo]."""
    return _DWConv.apply(x.contiguous(), w, int(C), int(stride))


class _PlaneBN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, C, eps, relu, stats_out):
        B, CC, H, W = x.shape
        Ch = CC // C
        mean = torch.empty(CC, dtype=torch.float32, device=x.device)
        var = torch.empty(CC, dtype=torch.float32, device=x.device)
        pcs = weight.stride(0) if weight is not None else 0
        common = (_p(weight), _p(bias), _i64(pcs), _p(mean), _p(var), _f(eps), _c.c_int(int(relu)))
        dims = (_c.c_int(B), _c.c_int(CC), _c.c_int(Ch), _c.c_int(H * W), _stream(x))
        rc = _fn("fa_plane_bn")(_c.c_int(0), _c.c_int(_bf(x)), _p(x), None, None, *common, None, *dims)
        _check(rc, "fa_plane_bn stats")
        y = torch.empty_like(x)
        rc = _fn("fa_plane_bn")(_c.c_int(1), _c.c_int(_bf(x)), _p(x), None, _p(y), *common, None, *dims)
        _check(rc, "fa_plane_bn apply")
        stats_out.append((mean.view(C, Ch), var.view(C, Ch), float(B * H * W)))
        ctx.save_for_backward(x, weight, bias, mean, var)
        ctx.cfg = (C, eps, relu)
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
        dims = (_c.c_int(B), _c.c_int(CC), _c.c_int(Ch), _c.c_int(H * W), _stream(x))
        rc = _fn("fa_plane_bn")(_c.c_int(2), _c.c_int(_bf(x)), _p(x), _p(gy), None, *common, _p(red), *dims)
        _check(rc, "fa_plane_bn bwd_reduce")
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            rc = _fn("fa_plane_bn")(_c.c_int(3), _c.c_int(_bf(x)), _p(x), _p(gy), _p(dx), *common, _p(red), *dims)
            _check(rc, "fa_plane_bn dx")
        rs = torch.rsqrt(var + eps)
        dg = (red[:, 1] * rs).view(C, Ch) if weight is not None else None
        db = red[:, 0].view(C, Ch) if bias is not None else None
        return dx, dg, db, None, None, None, None


def plane_batch_norm(x, weight, bias, C, eps, relu=False):
    """Training BN(+ReLU) of client-stacked x [B, C·Ch, H, W] with per-client affine [C, Ch] (or None).
    Returns (y, (mean [C, Ch], biased var [C, Ch], n)) — the statistics for the running-average update."""
    stats = []
    y = _PlaneBN.apply(x.contiguous(), weight, bias, int(C), float(eps), bool(relu), stats)
    return y, stats[0]


def plane_supported(x, weight, C) -> bool:
    return (x.is_cuda and x.dim() == 4 and x.dtype in (torch.float32, torch.bfloat16) and x.shape[1] % C == 0
            and (weight is None or (weight.dtype == torch.float32 and weight[0].is_contiguous())))
