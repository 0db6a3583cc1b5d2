"""Python entry points for the FL kernels (``csrc/fl_kernels.hip``).

Dispatch: CUDA(HIP) tensors → native kernel (mandatory on GPU: raises if the
library is missing); CPU tensors → the plain-PyTorch fp32 reference of the same
op (also the oracle the GPU tests compare against). ``FEDML_AMD_FORCE_TORCH=1``
forces the reference on GPU for A/B measurements only.
"""
import ctypes
import os

import torch

from . import _native

_c = ctypes
_FORCE_TORCH = os.environ.get("FEDML_AMD_FORCE_TORCH", "0") == "1"
_SIGS = {}


_SC = None   # stream-ordering checker (core/tracing/stream_check.py) when installed


def _p(t):
    if t is None:
        return None
    if _SC is not None and t.is_cuda:
        _SC.pending(t)
    return _c.c_void_p(t.data_ptr())


def _pr(t):
    """:func:`_p` for an operand the kernel only READS (the stream checker records a read, not a write)."""
    if t is None:
        return None
    if _SC is not None and t.is_cuda:
        _SC.pending(t, write=False)
    return _c.c_void_p(t.data_ptr())


def _stream(t):
    return _c.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def use_native(t: torch.Tensor) -> bool:
    return t.is_cuda and not _FORCE_TORCH


def _fn(name, restype=_c.c_int):
    lib = _native.lib(required=True)
    f = _SIGS.get(name)
    if f is None:
        f = getattr(lib, name)
        f.restype = restype
        _SIGS[name] = f
    return f


# Debug mode: FEDML_AMD_KERNEL_SYNC=1 synchronises after every native launch so an asynchronous
# device fault is attributed to the kernel that caused it (pair with AMD_SERIALIZE_KERNEL=3 to
# do the same for library kernels).
_KERNEL_SYNC = os.environ.get("FEDML_AMD_KERNEL_SYNC", "0") == "1"


def _check(rc, name):
    if _SC is not None:
        _SC.flush(name)
    if rc != 0:
        raise RuntimeError(f"{name} failed with HIP error {rc}")
    if _KERNEL_SYNC:
        import torch as _t
        try:
            _t.cuda.synchronize()
        except Exception as e:  # noqa: BLE001 - re-raise naming the kernel
            raise RuntimeError(f"device fault in {name}: {e}") from e


def _i64(v):
    return _c.c_int64(int(v))


def _f(v):
    return _c.c_float(float(v))


def _u64(v):
    return _c.c_uint64(int(v) & ((1 << 64) - 1))


# ----------------------------------------------------------------------------- K1
def weighted_sum(stack: torch.Tensor, w: torch.Tensor, out: torch.Tensor = None, beta: float = 0.0) -> torch.Tensor:
    """out = beta*out + Σ_c w[c]·stack[c]  for a [C, P] fp32/bf16 stack (fp32 result)."""
    assert stack.dim() == 2
    C, P = stack.shape
    if out is None:
        out = torch.empty(P, dtype=torch.float32, device=stack.device)
        beta = 0.0
    if use_native(stack):
        assert stack.stride(1) == 1 and stack.dtype in (torch.float32, torch.bfloat16)
        w = w.to(device=stack.device, dtype=torch.float32).contiguous()
        rc = _fn("fa_weighted_sum")(_p(stack), _c.c_int(stack.dtype == torch.bfloat16), _i64(stack.stride(0)),
                                     _c.c_int(C), _p(w), _p(out), _i64(P), _f(beta), _stream(stack))
        _check(rc, "fa_weighted_sum")
        return out
    res = (w.to(torch.float32).view(C, 1) * stack.to(torch.float32)).sum(0)
    if beta != 0.0:
        res = res + beta * out
    out.copy_(res)
    return out


def broadcast_rows_(dst: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
    """dst[c, :] = src for every row of the [C, P] fp32 stack ``dst`` (unit inner stride) — one vectorised
    launch (torch's copy of an expanded source splits a > 2^31-element stack into dozens of strided launches)."""
    C, P = dst.shape
    if use_native(dst) and dst.dtype == torch.float32 and src.dtype == torch.float32 and dst.stride(1) == 1 \
            and src.is_contiguous() and src.numel() == P:
        _check(_fn("fa_broadcast_rows")(_p(dst), _p(src), _c.c_int(C), _i64(P), _i64(dst.stride(0)), _stream(dst)),
               "fa_broadcast_rows")
        return dst
    dst.copy_(src.reshape(1, P).expand(C, P))
    return dst


class ZeroSegments:
    """Column ranges [(off, len)] of a [C, P] fp32 stack zeroed by one launch (``fa_zero_segments``); the
    table lives on the device (built once, replayable from a captured graph)."""

    def __init__(self, segs, device):
        self.segs = [(int(o), int(n)) for o, n in segs if n > 0]
        flat = [v for seg in self.segs for v in seg]
        self.table = torch.tensor(flat or [0, 0], dtype=torch.int64, device=device)
        self.max_len = max((n for _, n in self.segs), default=0)

    def __call__(self, stack: torch.Tensor):
        if use_native(stack) and stack.dtype == torch.float32 and stack.stride(1) == 1:
            _check(_fn("fa_zero_segments")(_p(stack), _i64(stack.stride(0)), _c.c_int(stack.shape[0]), _p(self.table),
                                           _c.c_int(len(self.segs)), _i64(self.max_len), _stream(stack)),
                   "fa_zero_segments")
        else:
            for o, n in self.segs:
                stack[:, o:o + n].zero_()
        return stack


def complement_segments(P: int, taken):
    """The column ranges of [0, P) not covered by ``taken`` [(off, len)]."""
    out, pos = [], 0
    for o, n in sorted(taken):
        if o > pos:
            out.append((pos, o - pos))
        pos = max(pos, o + n)
    if pos < P:
        out.append((pos, P - pos))
    return out


def weighted_average(stack: torch.Tensor, counts) -> torch.Tensor:
    """FedAvg: Σ_c (n_c / Σn) · stack[c]."""
    w = torch.as_tensor(counts, dtype=torch.float64)
    w = (w / w.sum()).to(torch.float32)
    return weighted_sum(stack, w.to(stack.device))


def subset_aggregate(W: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
    """OUT[S, P] = W[S, C] @ X[C, P]  (exact-fp32 MFMA on GPU)."""
    S, C = W.shape
    P = X.shape[1]
    if use_native(X):
        W = W.to(device=X.device, dtype=torch.float32).contiguous()
        X = X.to(torch.float32)
        out = torch.zeros(S, P, dtype=torch.float32, device=X.device)
        for c0 in range(0, C, 64):
            c1 = min(C, c0 + 64)
            part = out if c0 == 0 else torch.empty_like(out)
            rc = _fn("fa_subset_aggregate")(_p(W[:, c0:c1].contiguous()), _c.c_int(S), _c.c_int(c1 - c0),
                                             _p(X[c0:c1]), _i64(X.stride(0)), _i64(P), _p(part), _i64(P),
                                             _stream(X))
            _check(rc, "fa_subset_aggregate")
            if c0:
                out += part
        return out
    return W.to(torch.float32) @ X.to(torch.float32)


# ----------------------------------------------------------------------------- K2
def sgd_step(param, grad, lr, weight_decay=0.0, momentum=0.0, mom_buf=None, dampening=0.0, nesterov=False,
             mu=0.0, global_ref=None, first_step=False, active=None, lr_scale=None):
    """In-place fused SGD over a [C, P] stack (torch.optim.SGD semantics; FedProx term μ(w − w_g))."""
    C, P = param.shape
    if use_native(param):
        assert param.dtype == torch.float32 and param.stride(1) == 1 and grad.stride(1) == 1
        assert grad.stride(0) == param.stride(0)
        rc = _fn("fa_sgd_step")(_p(param), _p(grad), _c.c_int(grad.dtype == torch.bfloat16),
                                _p(mom_buf if momentum != 0.0 else None), _p(global_ref), _c.c_int(C), _i64(P),
                                _i64(param.stride(0)), _f(lr), _f(weight_decay), _f(momentum), _f(dampening),
                                _c.c_int(int(nesterov)), _f(mu), _c.c_int(int(first_step)), _p(active),
                                _p(lr_scale), _stream(param))
        _check(rc, "fa_sgd_step")
        return param
    g = grad.to(torch.float32)
    if mu != 0.0:
        g = g + mu * (param - global_ref.view(1, -1))
    if weight_decay != 0.0:
        g = g + weight_decay * param
    d = g
    on = torch.ones(C, 1, dtype=torch.bool) if active is None else (active.view(C, 1) > 0)
    if momentum != 0.0:
        nb = g if first_step else momentum * mom_buf + (1.0 - dampening) * g
        mom_buf.copy_(torch.where(on, nb, mom_buf))
        d = g + momentum * mom_buf if nesterov else mom_buf
    scale = torch.ones(C, 1, dtype=torch.float32) if active is None else active.view(C, 1).to(torch.float32)
    if lr_scale is not None:
        scale = scale * lr_scale.view(1, 1)
    # inactive clients are skipped entirely (their gradients may hold garbage), as in the kernel
    param.copy_(torch.where(scale > 0, param - lr * scale * d, param))
    return param


def adam_step(param, grad, exp_avg, exp_avg_sq, step, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0,
              amsgrad=False, max_exp_avg_sq=None, decoupled=False, active=None, shadow=None):
    """In-place fused Adam/AMSGrad/AdamW over a [C, P] stack; ``step`` is a [C] fp32 device tensor
    holding the (already incremented) step count of each client. ``shadow`` ([C, P] bf16, same
    strides): also written with bf16(updated param) in the same pass (inactive clients untouched)."""
    C, P = param.shape
    if use_native(param):
        assert shadow is None or (shadow.dtype == torch.bfloat16 and shadow.stride() == param.stride())
        rc = _fn("fa_adam_step")(_p(param), _p(grad), _c.c_int(grad.dtype == torch.bfloat16), _p(exp_avg),
                                 _p(exp_avg_sq), _p(max_exp_avg_sq if amsgrad else None), _p(step), _c.c_int(C),
                                 _i64(P), _i64(param.stride(0)), _f(lr), _f(beta1), _f(beta2), _f(eps),
                                 _f(weight_decay), _c.c_int(int(decoupled)), _p(active), _p(shadow), _stream(param))
        _check(rc, "fa_adam_step")
        return param
    # Same contract as the HIP kernel: an inactive client (active[c] == 0) is skipped ENTIRELY — its
    # parameters, moments, AMSGrad maximum and shadow row keep their values (no weight decay either).
    on = (active.view(C, 1) != 0) if active is not None else torch.ones(C, 1, dtype=torch.bool, device=param.device)
    g = grad.to(torch.float32)
    t = step.view(C, 1).to(torch.float32)
    p = param
    if weight_decay != 0.0:
        if decoupled:
            p = param * (1 - lr * weight_decay)
        else:
            g = g + weight_decay * param
    # first step (t ≤ 1): the moments start from zero whatever the buffers hold (the native kernel never reads
    # them then; callers need not reset them between rounds)
    fresh = t <= 1
    m1 = torch.where(fresh, 0.0, exp_avg) * beta1 + (1 - beta1) * g
    m2 = torch.where(fresh, 0.0, exp_avg_sq) * beta2 + (1 - beta2) * g * g
    bc1 = 1 - beta1 ** t
    bc2 = 1 - beta2 ** t
    if amsgrad:
        vm = torch.where(fresh, m2, torch.maximum(max_exp_avg_sq, m2))
        den = vm.sqrt() / bc2.sqrt() + eps
        max_exp_avg_sq.copy_(torch.where(on, vm, max_exp_avg_sq))
    else:
        den = m2.sqrt() / bc2.sqrt() + eps
    exp_avg.copy_(torch.where(on, m1, exp_avg))
    exp_avg_sq.copy_(torch.where(on, m2, exp_avg_sq))
    param.copy_(torch.where(on, p - (lr / bc1) * m1 / den, param))
    if shadow is not None:
        shadow.copy_(torch.where(on, param.to(torch.bfloat16), shadow))
    return param


# ----------------------------------------------------------------------------- K10
_FEDOPT_IDS = {"sgd": 0, "fedavgm": 0, "adam": 1, "fedadam": 1, "yogi": 2, "fedyogi": 2, "adagrad": 3,
               "fedadagrad": 3}


def fednova_server_step(glob, wsum, S, buf=None, gmf=0.0, lr=1.0, first=False):
    """FedNova server update in place on ``glob`` (flat fp32 [P]) from the all-reduced coefficient-weighted
    client sum ``wsum`` [P] and ``S`` = Σ coef (a 1-element device tensor): cum = S·glob − wsum; glob −= cum,
    or with server momentum ``gmf``: buf = (first ? 0 : gmf·buf) + cum/lr, glob −= lr·buf (csrc K11)."""
    P = glob.numel()
    if gmf and buf is None:
        raise ValueError("fednova_server_step: gmf > 0 needs a momentum buffer")
    if use_native(glob):
        rc = _fn("fa_fednova_server_step")(_p(glob), _p(wsum), _p(S), _p(buf), _i64(P), _f(gmf), _f(lr),
                                           _c.c_int(int(bool(first))), _stream(glob))
        _check(rc, "fa_fednova_server_step")
        return glob
    cum = S.view(()) * glob - wsum
    if gmf:
        if first:
            buf.copy_(cum / lr)
        else:
            buf.mul_(gmf).add_(cum, alpha=1.0 / lr)
        glob.sub_(lr * buf)
    else:
        glob.sub_(cum)
    return glob


def fedopt_step(stack, w, glob, opt="sgd", lr=1.0, beta1=0.9, beta2=0.99, eps=1e-3, momentum=0.0, nesterov=False,
                state1=None, state2=None, step=1, first_step=False):
    """Fused FedOpt server update: avg = Σ w_c stack_c; g = glob − avg; glob ← ServerOpt(glob, g)."""
    C, P = stack.shape
    oid = _FEDOPT_IDS[opt.lower()]
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    if use_native(stack):
        w = w.to(device=stack.device, dtype=torch.float32).contiguous()
        rc = _fn("fa_fedopt_step")(_p(stack), _i64(stack.stride(0)), _c.c_int(C), _p(w), _p(glob), _p(state1),
                                   _p(state2), _i64(P), _c.c_int(oid), _f(lr), _f(beta1), _f(beta2), _f(eps),
                                   _f(bc1), _f(bc2), _f(momentum), _c.c_int(int(nesterov)),
                                   _c.c_int(int(first_step)), _stream(stack))
        _check(rc, "fa_fedopt_step")
        return glob
    avg = (w.view(C, 1).to(torch.float32) * stack).sum(0)
    g = glob - avg
    if oid == 0:
        d = g
        if momentum != 0.0:
            if first_step:
                state1.copy_(g)
            else:
                state1.mul_(momentum).add_(g)
            d = g + momentum * state1 if nesterov else state1
        glob.sub_(lr * d)
    elif oid in (1, 2):
        state1.mul_(beta1).add_(g, alpha=1 - beta1)
        if oid == 1:
            state2.mul_(beta2).addcmul_(g, g, value=1 - beta2)
        else:
            g2 = g * g
            sgn = torch.where(state2 - g2 < 0, -torch.ones_like(g2), torch.ones_like(g2))
            state2.sub_((1 - beta2) * g2 * sgn)
        glob.sub_(lr * (state1 / bc1) / ((state2.clamp_min(0) / bc2).sqrt() + eps))
    else:
        state2.add_(g * g)
        glob.sub_(lr * g / (state2.sqrt() + eps))
    return glob


# ----------------------------------------------------------------------------- K9
def client_sqnorm(stack, ref=None, mask=None):
    """[C] squared L2 norms of (stack_c − ref) over the masked coordinates (deterministic)."""
    C, P = stack.shape
    if use_native(stack):
        out = torch.empty(C, dtype=torch.float32, device=stack.device)
        partial = torch.empty(C * 64, dtype=torch.float32, device=stack.device)
        rc = _fn("fa_client_sqnorm")(_p(stack), _i64(stack.stride(0)), _c.c_int(C), _p(ref), _p(mask), _i64(P),
                                     _p(partial), _p(out), _stream(stack))
        _check(rc, "fa_client_sqnorm")
        return out
    d = stack - (ref.view(1, -1) if ref is not None else 0.0)
    if mask is not None:
        d = d * mask.view(1, -1).to(d.dtype)
    return (d.double() ** 2).sum(1).to(torch.float32)


def norm_diff_clip_(stack, ref, bound, mask=None, sqnorm=None):
    """stack_c ← ref + (stack_c − ref) / max(1, ‖stack_c − ref‖ / bound)  (in place)."""
    C, P = stack.shape
    if sqnorm is None:
        sqnorm = client_sqnorm(stack, ref, mask)
    if use_native(stack):
        rc = _fn("fa_norm_clip")(_p(stack), _i64(stack.stride(0)), _c.c_int(C), _p(ref), _p(mask), _p(sqnorm),
                                 _i64(P), _f(bound), _stream(stack))
        _check(rc, "fa_norm_clip")
        return stack
    scale = 1.0 / torch.clamp(sqnorm.sqrt() / bound, min=1.0)
    r = ref.view(1, -1) if ref is not None else torch.zeros(1, P, dtype=stack.dtype)
    new = r + (stack - r) * scale.view(C, 1)
    if mask is not None:
        m = mask.view(1, -1).bool()
        new = torch.where(m, new, stack)
    stack.copy_(new)
    return stack


def gaussian_noise_(x, stddev, seed=0, offset=0, mask=None):
    """x += stddev·N(0,1) (counter-based Philox on GPU; torch generator on CPU)."""
    if use_native(x):
        assert x.is_contiguous() and x.dtype == torch.float32
        rc = _fn("fa_gaussian_noise")(_p(x), _p(mask), _i64(x.numel()), _f(stddev), _u64(seed), _u64(offset),
                                      _stream(x))
        _check(rc, "fa_gaussian_noise")
        return x
    g = torch.Generator().manual_seed(int(seed) + int(offset))
    noise = torch.randn(x.shape, generator=g, dtype=torch.float32) * stddev
    if mask is not None:
        noise = noise * mask.view(x.shape).to(noise.dtype)
    x.add_(noise)
    return x


def coordinate_median(stack):
    """Coordinate-wise (lower) median over clients: [C, P] → [P]."""
    C, P = stack.shape
    if use_native(stack) and C <= 64:
        out = torch.empty(P, dtype=torch.float32, device=stack.device)
        rc = _fn("fa_coordinate_median")(_p(stack), _i64(stack.stride(0)), _c.c_int(C), _i64(P), _p(out),
                                         _stream(stack))
        _check(rc, "fa_coordinate_median")
        return out
    return torch.median(stack.to(torch.float32), dim=0).values


# ----------------------------------------------------------------------------- K15
def compress_accumulate(params, glob, residual_rows, weights, ids, method, seed, out):
    """One launch over the [C, P] client stack: out = Σ_c w_c·(glob + D(C(Δ_c + r_c))) with Δ_c =
    params[c] − glob, C = block-256 int8 (stochastic rounding keyed by (seed, client id, element)) or
    fp8-e4m3 quantisation, and the error-feedback rows r_c updated in place (``residual_rows``: list of
    C fp32 [P] tensors or None). ``weights`` [C] / ``ids`` [C] stay on the device (no host sync)."""
    mode = {"int8": 0, "fp8": 1}[method]
    C, P = params.shape[0], glob.numel()
    if not use_native(params):
        out.zero_()
        for c in range(C):
            r = residual_rows[c] if residual_rows is not None else None
            d = params[c] - glob
            back = torch.zeros_like(glob)
            if mode == 0:
                q, sc = quantize_int8(d, residual=r, stochastic=True, seed=seed * 1000003 + int(ids[c]))
                dequantize_int8_axpy(q, sc, 1.0, back)
            else:
                q, sc = quantize_fp8(d, residual=r)
                dequantize_fp8_axpy(q, sc, 1.0, back)
            out += float(weights[c]) * (glob + back)
        return out
    rows = torch.tensor([r.data_ptr() if r is not None else 0 for r in residual_rows] if residual_rows is not None
                        else [0] * C, dtype=torch.int64).to(params.device, non_blocking=True)
    rc = _fn("fa_compress_accumulate")(_p(params), _i64(params.stride(0)), _c.c_int(C), _p(glob), _p(rows),
                                       _p(weights.to(torch.float32).contiguous()), _p(ids.to(torch.int64).contiguous()),
                                       _p(out), _i64(P), _c.c_int(mode), _u64(seed), _stream(params))
    _check(rc, "fa_compress_accumulate")
    return out


def quantize_int8(x, residual=None, stochastic=True, seed=0):
    """Block-256 int8 quantisation with optional stochastic rounding and error feedback.
    Returns (q int8 [n], scales f32 [ceil(n/256)]); ``residual`` (if given) is updated to x+r−deq."""
    n = x.numel()
    nb = (n + 255) // 256
    if use_native(x):
        q = torch.empty(n, dtype=torch.int8, device=x.device)
        s = torch.empty(nb, dtype=torch.float32, device=x.device)
        rc = _fn("fa_quant_int8")(_p(x), _p(residual), _p(q), _p(s), _i64(n), _c.c_int(int(stochastic)), _u64(seed),
                                  _stream(x))
        _check(rc, "fa_quant_int8")
        return q, s
    v = x.reshape(-1).to(torch.float32) + (residual.reshape(-1) if residual is not None else 0.0)
    pad = nb * 256 - n
    vp = torch.nn.functional.pad(v, (0, pad)).view(nb, 256)
    amax = vp.abs().amax(1)
    scale = torch.where(amax > 0, amax / 127.0, torch.ones_like(amax))
    t = vp / scale.view(-1, 1)
    if stochastic:
        g = torch.Generator().manual_seed(int(seed))
        t = torch.floor(t + torch.rand(t.shape, generator=g))
    else:
        t = torch.round(t)
    t = t.clamp(-127, 127)
    q = t.reshape(-1)[:n].to(torch.int8)
    if residual is not None:
        residual.copy_((v - (t * scale.view(-1, 1)).reshape(-1)[:n]).view_as(residual))
    return q, scale


def dequantize_int8_axpy(q, scales, w, acc):
    """acc += w · dequant(q)."""
    n = q.numel()
    if use_native(acc):
        rc = _fn("fa_dequant_int8_axpy")(_p(q), _p(scales), _f(w), _p(acc), _i64(n), _stream(acc))
        _check(rc, "fa_dequant_int8_axpy")
        return acc
    s = scales.repeat_interleave(256)[:n]
    acc.add_(w * q.to(torch.float32) * s)
    return acc


def quantize_fp8(x, residual=None):
    """Block-256 OCP fp8 e4m3fn quantisation (+ optional error feedback). Returns (q uint8, scales)."""
    n = x.numel()
    nb = (n + 255) // 256
    if use_native(x):
        q = torch.empty(n, dtype=torch.uint8, device=x.device)
        s = torch.empty(nb, dtype=torch.float32, device=x.device)
        rc = _fn("fa_quant_fp8")(_p(x), _p(residual), _p(q), _p(s), _i64(n), _stream(x))
        _check(rc, "fa_quant_fp8")
        return q, s
    v = x.reshape(-1).to(torch.float32) + (residual.reshape(-1) if residual is not None else 0.0)
    pad = nb * 256 - n
    vp = torch.nn.functional.pad(v, (0, pad)).view(nb, 256)
    amax = vp.abs().amax(1)
    scale = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
    inv = 1.0 / scale   # multiply by the reciprocal, exactly as the HIP kernel does
    t = (vp * inv.view(-1, 1)).clamp(-448, 448).to(torch.float8_e4m3fn)
    q = t.reshape(-1)[:n].view(torch.uint8)
    if residual is not None:
        back = t.to(torch.float32) * scale.view(-1, 1)
        residual.copy_((v - back.reshape(-1)[:n]).view_as(residual))
    return q, scale


def dequantize_fp8_axpy(q, scales, w, acc):
    n = q.numel()
    if use_native(acc):
        rc = _fn("fa_dequant_fp8_axpy")(_p(q), _p(scales), _f(w), _p(acc), _i64(n), _stream(acc))
        _check(rc, "fa_dequant_fp8_axpy")
        return acc
    s = scales.repeat_interleave(256)[:n]
    acc.add_(w * q.view(torch.float8_e4m3fn).to(torch.float32) * s)
    return acc


class _TopkScratch:
    cache = {}
    batched = {}   # (device, C) → (state [C·8], hist [C·2048]) of topk_compress_accumulate

    @classmethod
    def get(cls, device):
        key = str(device)
        if key not in cls.cache:
            cls.cache[key] = (torch.zeros(8, dtype=torch.int32, device=device),
                              torch.zeros(2048, dtype=torch.int32, device=device))
        return cls.cache[key]


def topk_abs(x, k, residual=None):
    """Exact top-k of |x| (radix select on device). Returns (idx int32 [k], val f32 [k]) — order unspecified.
    ``residual`` (if given) receives x with the selected entries zeroed (error feedback)."""
    n = x.numel()
    k = int(min(max(k, 1), n))
    xf = x.reshape(-1)
    if use_native(x):
        idx = torch.empty(k, dtype=torch.int32, device=x.device)
        val = torch.empty(k, dtype=torch.float32, device=x.device)
        state, hist = _TopkScratch.get(x.device)
        rc = _fn("fa_topk_abs")(_p(xf), _i64(n), _i64(k), _p(state), _p(hist), _p(idx), _p(val),
                                _p(residual.reshape(-1) if residual is not None else None), _stream(x))
        _check(rc, "fa_topk_abs")
        return idx, val
    _, i = torch.topk(xf.abs(), k)
    val = xf[i].to(torch.float32)
    if residual is not None:
        r = xf.to(torch.float32).clone()
        r[i] = 0.0
        residual.copy_(r.view_as(residual))
    return i.to(torch.int32), val


def topk_compress_accumulate(params, glob, residual_rows, weights, k, out):
    """All C clients of the [C, P] stack in one batched radix select (8 launches for any C): client c's
    update Δ_c = params[c] − glob + r_c keeps its k largest |Δ_c| entries (exact, ties cut by count), the rest
    becomes its new residual r_c (``residual_rows``: list of C fp32 [P] rows or None entries, or None), and
    out = Σ_c w_c·(glob + topk(Δ_c)). Slots with w_c = 0 are skipped (their rows untouched). ``weights``
    stays on the device."""
    C, P = params.shape[0], glob.numel()
    k = int(min(max(int(k), 1), P))
    if use_native(params) and P % 4 == 0 and params.stride(0) % 4 == 0:
        key = (str(params.device), C)
        sc = _TopkScratch.batched.get(key)
        if sc is None:
            sc = _TopkScratch.batched[key] = (torch.zeros(C * 8, dtype=torch.int32, device=params.device),
                                              torch.zeros(C * 2048, dtype=torch.int32, device=params.device))
        rows = torch.tensor([r.data_ptr() if r is not None else 0 for r in residual_rows]
                            if residual_rows is not None else [0] * C, dtype=torch.int64).to(params.device,
                                                                                             non_blocking=True)
        rc = _fn("fa_topk_compress_accumulate")(_p(params), _i64(params.stride(0)), _c.c_int(C), _p(glob), _p(rows),
                                                _p(weights.to(torch.float32).contiguous()), _i64(P), _i64(k),
                                                _p(sc[0]), _p(sc[1]), _p(out), _stream(params))
        _check(rc, "fa_topk_compress_accumulate")
        return out
    w_host = weights.to(torch.float32).tolist()
    acc = torch.zeros(P, dtype=torch.float32, device=params.device)
    for c, wc in enumerate(w_host):
        if wc == 0.0:
            continue
        r = residual_rows[c] if residual_rows is not None else None
        d = params[c].to(torch.float32) - glob
        if r is not None:
            d = d + r
        idx, val = topk_abs(d, k, residual=r)
        acc.index_add_(0, idx.long(), wc * val)
    out.copy_(acc + float(sum(w_host)) * glob)
    return out


def scatter_axpy(idx, val, w, acc):
    """acc[idx] += w · val (indices unique within one call)."""
    if use_native(acc):
        rc = _fn("fa_scatter_axpy")(_p(idx), _p(val), _i64(idx.numel()), _f(w), _p(acc), _stream(acc))
        _check(rc, "fa_scatter_axpy")
        return acc
    acc.index_add_(0, idx.long(), w * val.to(acc.dtype))
    return acc


# ----------------------------------------------------------------------------- K7
def softmax_xent_fwd_bwd(logits, labels, class_weight=None, row_scale=None, ignore_index=-100, need_grad=True):
    """Fused per-row CE: returns (loss_rows [R], dlogits [R, K] or None) where
    dlogits = cw[y]·row_scale·(softmax − onehot)."""
    R, K = logits.shape
    if use_native(logits):
        assert logits.is_contiguous() and logits.dtype in (torch.float32, torch.bfloat16)
        loss = torch.empty(R, dtype=torch.float32, device=logits.device)
        dz = torch.empty_like(logits) if need_grad else None
        lab = labels.to(torch.int64).contiguous()
        rc = _fn("fa_softmax_xent")(_p(logits), _c.c_int(logits.dtype == torch.bfloat16), _p(lab),
                                    _p(class_weight), _p(row_scale), _p(dz), _p(loss), _i64(R), _c.c_int(K),
                                    _i64(ignore_index), _stream(logits))
        _check(rc, "fa_softmax_xent")
        return loss, dz
    z = logits.to(torch.float32)
    lab = labels.to(torch.int64)
    ign = (lab == ignore_index) | (lab < 0) | (lab >= K)
    safe = lab.clamp(0, K - 1)
    lse = torch.logsumexp(z, 1)
    cw = class_weight[safe] if class_weight is not None else torch.ones(R)
    cw = torch.where(ign, torch.zeros_like(cw), cw)
    loss = cw * (lse - z.gather(1, safe.view(-1, 1)).squeeze(1))
    dz = None
    if need_grad:
        p = torch.softmax(z, 1)
        p[torch.arange(R), safe] -= 1.0
        rs = row_scale if row_scale is not None else torch.ones(R)
        dz = (p * (cw * rs).view(-1, 1)).to(logits.dtype)
    return loss, dz


class FusedCrossEntropy(torch.autograd.Function):
    """Autograd wrapper: mean CE per group of rows (per virtual client) summed over groups."""

    @staticmethod
    def forward(ctx, logits, labels, row_scale, class_weight):
        loss_rows, dz = softmax_xent_fwd_bwd(logits, labels, class_weight, row_scale, need_grad=True)
        ctx.save_for_backward(dz)
        return (loss_rows * row_scale).sum()

    @staticmethod
    def backward(ctx, g):
        (dz,) = ctx.saved_tensors
        return dz * g.to(dz.dtype), None, None, None


# ----------------------------------------------------------------------------- K8
def confusion_matrix(logits, labels, num_groups=1, rows_per_group=None):
    """[G, K, K] int32 counts of (label, argmax) per group of rows."""
    R, K = logits.shape
    rpg = rows_per_group or max(1, R // max(1, num_groups))
    if use_native(logits):
        cm = torch.zeros(num_groups, K, K, dtype=torch.int32, device=logits.device)
        rc = _fn("fa_confusion")(_p(logits.contiguous()), _c.c_int(logits.dtype == torch.bfloat16),
                                 _p(labels.to(torch.int64).contiguous()), _p(cm), _i64(R), _c.c_int(K), _i64(rpg),
                                 _stream(logits))
        _check(rc, "fa_confusion")
        return cm
    pred = logits.to(torch.float32).argmax(1)
    g = torch.arange(R) // rpg
    flat = (g * K + labels.long()) * K + pred
    return torch.bincount(flat, minlength=num_groups * K * K).view(num_groups, K, K).to(torch.int32)


def eval_stats(logits, labels, groups=None, num_groups=1, with_classes=False, sums=None, cls=None):
    """Accumulate evaluation statistics of a logits block [R, K] into per-group buffers (K8b):
    ``sums`` [G, 3] fp32 = (correct, Σ cross-entropy, rows) and, with ``with_classes``, ``cls`` [G, 3, K]
    int32 = (true positives, actual, predicted) per class. ``groups`` [R] int32 group of each row (None: 0);
    rows with a label outside [0, K) or a negative group are skipped. Returns (sums, cls)."""
    R, K = logits.shape
    dev = logits.device
    if sums is None:
        sums = torch.zeros(num_groups, 3, dtype=torch.float32, device=dev)
    if with_classes and cls is None:
        cls = torch.zeros(num_groups, 3, K, dtype=torch.int32, device=dev)
    if R == 0:
        return sums, cls
    lab = labels.reshape(-1).to(torch.int64)
    grp = None if groups is None else groups.reshape(-1).to(torch.int32)
    if use_native(logits):
        rc = _fn("fa_eval_stats")(_pr(logits.contiguous()), _c.c_int(logits.dtype == torch.bfloat16),
                                  _pr(lab.contiguous()), _pr(None if grp is None else grp.contiguous()), _p(sums),
                                  _p(cls if with_classes else None), _i64(R), _c.c_int(K), _stream(logits))
        _check(rc, "fa_eval_stats")
        return sums, cls
    z = logits.to(torch.float32)
    g = torch.zeros(R, dtype=torch.int64, device=dev) if grp is None else grp.to(torch.int64)
    ok = (lab >= 0) & (lab < K) & (g >= 0)
    z, lab, g = z[ok], lab[ok], g[ok]
    pred = z.argmax(1)
    loss = torch.nn.functional.cross_entropy(z, lab, reduction="none")
    G = sums.shape[0]
    sums[:, 0].add_(torch.bincount(g, weights=(pred == lab).to(torch.float32), minlength=G).to(sums.dtype))
    sums[:, 1].add_(torch.bincount(g, weights=loss, minlength=G).to(sums.dtype))
    sums[:, 2].add_(torch.bincount(g, minlength=G).to(sums.dtype))
    if with_classes:
        hit = (pred == lab).to(torch.int64)
        c = cls.view(G, 3, K)
        c[:, 0].add_(torch.bincount(g * K + lab, weights=hit.to(torch.float64), minlength=G * K).view(G, K)
                     .to(torch.int32))
        c[:, 1].add_(torch.bincount(g * K + lab, minlength=G * K).view(G, K).to(torch.int32))
        c[:, 2].add_(torch.bincount(g * K + pred, minlength=G * K).view(G, K).to(torch.int32))
    return sums, cls


def cast_bf16(x, out=None):
    if use_native(x):
        out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device) if out is None else out
        rc = _fn("fa_cast_bf16")(_p(x), _p(out), _i64(x.numel()), _stream(x))
        _check(rc, "fa_cast_bf16")
        return out
    r = x.to(torch.bfloat16)
    if out is not None:
        out.copy_(r)
        return out
    return r


# ----------------------------------------------------------------------------- K13
def _mod_matmul_ref(A, B, p):
    A = A.to(torch.int64).remainder(p)
    B2 = B.reshape(B.shape[0], -1).to(torch.int64).remainder(p)
    out = torch.zeros(A.shape[0], B2.shape[1], dtype=torch.int64, device=B.device)
    for k in range(A.shape[1]):
        out = (out + (A[:, k:k + 1] * B2[k:k + 1]) % p) % p
    return out


def mod_matmul(A: torch.Tensor, B: torch.Tensor, p: int) -> torch.Tensor:
    """(A @ B) mod p on int64 residues (A: [M,K], B: [K, ...]); exact for p < 2^31."""
    shp = (A.shape[0],) + tuple(B.shape[1:])
    if use_native(B):
        A_ = A.to(device=B.device, dtype=torch.int64).remainder(p).contiguous()
        B_ = B.to(torch.int64).reshape(B.shape[0], -1).contiguous()
        out = torch.empty(A_.shape[0], B_.shape[1], dtype=torch.int64, device=B.device)
        rc = _fn("fa_mod_matmul")(_p(A_), _p(B_), _p(out), _c.c_int(A_.shape[0]), _c.c_int(A_.shape[1]),
                                  _i64(B_.shape[1]), _i64(p), _stream(B))
        _check(rc, "fa_mod_matmul")
        return out.reshape(shp)
    return _mod_matmul_ref(A, B, p).reshape(shp)


def mod_sum(X: torch.Tensor, p: int) -> torch.Tensor:
    """Σ_c X[c] mod p over residues (X: [C, ...])."""
    if use_native(X):
        X_ = X.to(torch.int64).contiguous()
        out = torch.empty(X_.shape[1:], dtype=torch.int64, device=X.device)
        rc = _fn("fa_mod_sum")(_p(X_), _p(out), _c.c_int(X_.shape[0]), _i64(out.numel()), _i64(p), _stream(X))
        _check(rc, "fa_mod_sum")
        return out
    acc = torch.zeros(X.shape[1:], dtype=torch.int64, device=X.device)
    for c in range(X.shape[0]):
        acc = (acc + X[c]) % p
    return acc


# ----------------------------------------------------------------------------- K16
def _philox4x32(c0, c1, c2, c3, k0, k1):
    """Host twin of common.h's Philox4x32-10 (used by the CPU reference of ``augment``)."""
    M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
    m = 0xFFFFFFFF
    for _ in range(10):
        p0, p1 = M0 * c0, M1 * c2
        hi0, lo0, hi1, lo1 = p0 >> 32, p0 & m, p1 >> 32, p1 & m
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & m, lo1, (hi0 ^ c3 ^ k1) & m, lo0
        k0, k1 = (k0 + W0) & m, (k1 + W1) & m
    return c0, c1, c2, c3


def augment(x, seed=0, sample_ids=None, pad=4, cutout=16, flip=True, mean=None, std=None):
    """RandomCrop(pad) + HorizontalFlip + Cutout + Normalize of a [B, C, H, W] fp32 batch (fused
    HIP kernel on GPU; per-sample Philox randomness keyed by (seed, sample id))."""
    B, C, H, W = x.shape
    mean_t = torch.as_tensor(mean, dtype=torch.float32, device=x.device) if mean is not None else None
    inv_t = (1.0 / torch.as_tensor(std, dtype=torch.float32, device=x.device)) if std is not None else None
    if use_native(x):
        xin = x.contiguous().float()
        out = torch.empty_like(xin)
        ids = sample_ids.to(device=x.device, dtype=torch.int64).contiguous() if sample_ids is not None else None
        rc = _fn("fa_augment")(_p(xin), _p(out), _p(ids), _c.c_int(B), _c.c_int(C), _c.c_int(H), _c.c_int(W),
                               _c.c_int(pad), _c.c_int(cutout), _c.c_int(int(flip)), _p(mean_t), _p(inv_t),
                               _c.c_uint32(seed & 0xFFFFFFFF), _stream(x))
        _check(rc, "fa_augment")
        return out
    out = torch.empty_like(x, dtype=torch.float32)
    ids = sample_ids.tolist() if sample_ids is not None else list(range(B))
    for b in range(B):
        sid = int(ids[b])
        r = _philox4x32(sid & 0xFFFFFFFF, (sid >> 32) & 0xFFFFFFFF, 0x41554721, 0, seed & 0xFFFFFFFF, 0x9E3779B9)
        dy = (r[0] % (2 * pad + 1)) - pad if pad else 0
        dx = (r[1] % (2 * pad + 1)) - pad if pad else 0
        fl = bool(flip and (r[2] & 1))
        shifted = torch.zeros_like(x[b], dtype=torch.float32)
        # out[oh, ow] = src[oh+dy, flip(ow)+dx]: crop offset applies in the unflipped frame
        src = x[b].float()
        ow = torch.arange(W)
        sw0 = (W - 1 - ow) if fl else ow
        for oh in range(H):
            sh = oh + dy
            if 0 <= sh < H:
                sw = sw0 + dx
                ok = (sw >= 0) & (sw < W)
                shifted[:, oh, ok] = src[:, sh, sw[ok]]
        if cutout:
            cy, cx = r[3] % H, (r[3] >> 16) % W
            h = cutout // 2
            shifted[:, max(0, cy - h):max(0, cy + h), max(0, cx - h):max(0, cx + h)] = 0
        if mean_t is not None:
            shifted = (shifted - mean_t.view(-1, 1, 1)) * inv_t.view(-1, 1, 1)
        out[b] = shifted
    return out


# ----------------------------------------------------------------------------- conv weight shadow
class ShadowSeg(ctypes.Structure):
    _fields_ = [("off", ctypes.c_int64), ("O", ctypes.c_int), ("I", ctypes.c_int), ("KH", ctypes.c_int),
                ("KW", ctypes.c_int)]


def pack_conv_shadow(params, shadow, segs_dev, nseg, max_n):
    """bf16 OHWI (channels-last) copies of the conv weights of a [C, P] fp32 arena into the same slots
    of a [C, P] bf16 arena (``segs_dev``: uint8 device tensor of ``ShadowSeg`` records)."""
    C = params.shape[0]
    rc = _fn("fa_pack_conv_shadow")(_p(params), _i64(params.stride(0)), _p(shadow), _i64(shadow.stride(0)),
                                    _p(segs_dev), _c.c_int(nseg), _c.c_int(max_n), _c.c_int(C), _stream(params))
    _check(rc, "fa_pack_conv_shadow")
