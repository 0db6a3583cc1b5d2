"""Autograd ops over the transformer HIP kernels (``csrc/transformer_kernels.hip``).

* :func:`layer_norm` — LN(res + dropout(h)) with per-client gamma/beta ``[C, d]`` (rows of client c
  are ``[c·R_c, (c+1)·R_c)``); backward gives dh (dropout-masked), dres, dgamma, dbeta.
* :func:`gelu` — exact (erf) GELU.
* :func:`attention` — softmax(q·kᵀ/√64 + key mask)·v per (row-group, head) for S ≤ 256 and head
  dim 64, with attention-probability dropout; q/k/v/o are token-major ``[CB·S, H·64]``.

CUDA tensors run the kernels at the tensor's storage precision: bf16 (``csrc/transformer_kernels.hip``,
``bgemm_kernels.hip``) or fp32 — the reference's training precision — (``csrc/tf_f32_kernels.hip``:
exact ``v_mfma_f32_16x16x4_f32`` products, or split-bf16 ones under ``fp32_mma: bf16x3``), fp32
statistics either way. CPU tensors run the plain-PyTorch fp32 reference of the same math — the same
hash-based dropout mask included — which is also the oracle of ``tests/test_transformer_kernels_gpu.py``.
"""
import contextlib
import ctypes as _c
import math

import torch

from .fl_ops import _check, _f, _fn, _i64, _p, _stream, use_native

_M32 = 0xFFFFFFFF


def _sfx(t: torch.Tensor) -> str:
    """Kernel-name suffix of a storage dtype: fp32 tensors run the ``_f32`` kernels."""
    if t.dtype == torch.float32:
        return "_f32"
    assert t.dtype == torch.bfloat16, f"transformer kernels take bf16 or fp32, got {t.dtype}"
    return ""


def _thr(p: float) -> int:
    return min(_M32, int(round(float(p) * 4294967296.0))) if p > 0 else 0


def _fmix32(h: torch.Tensor) -> torch.Tensor:
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & _M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & _M32
    return h ^ (h >> 16)


def dropout_keep(seed: int, a: torch.Tensor, b: torch.Tensor, p: float) -> torch.Tensor:
    """Keep mask of the kernels' counter-hash dropout: fmix32(fmix32(a ^ seed) + b·φ) ≥ p·2³²."""
    a = a.to(torch.int64) & _M32
    b = b.to(torch.int64) & _M32
    h = _fmix32((_fmix32(a ^ (int(seed) & _M32)) + b * 0x9E3779B1) & _M32)
    return h >= _thr(p)


# ------------------------------------------------------------------------------------------- LN
def _ct(t):
    """Compute dtype of the references: fp32, or fp64 for fp64 inputs (the kernels' numerics oracle)."""
    return torch.float64 if t.dtype == torch.float64 else torch.float32


def _ln_ref(h, res, gamma, beta, eps, p, seed, rpc):
    R, d = h.shape
    ct = _ct(h)
    x = h.to(ct)
    if p > 0:
        keep = dropout_keep(seed, torch.arange(R, device=h.device).view(R, 1),
                            torch.arange(d, device=h.device).view(1, d), p)
        x = torch.where(keep, x / (1.0 - p), torch.zeros_like(x))
    if res is not None:
        x = x + res.to(ct)
    if (res is not None or p > 0) and h.dtype == torch.bfloat16:
        x = x.to(torch.bfloat16).float()
    C = R // rpc
    xc = x.view(C, rpc, d)
    mu = xc.mean(-1, keepdim=True)
    var = ((xc - mu) ** 2).mean(-1, keepdim=True)
    y = (xc - mu) * torch.rsqrt(var + eps) * gamma.view(C, 1, d).to(ct) + beta.view(C, 1, d).to(ct)
    return y.view(R, d).to(h.dtype)


def _client_rows(gamma, beta):
    """(γ, β, client stride) for the LN kernels: per-client fp32 rows read in place when they are arena views
    (contiguous rows, a common 16-B aligned client stride), else a dense [C, d] copy."""
    if (gamma.dtype == torch.float32 and beta.dtype == torch.float32 and gamma.dim() == 2 and gamma[0].is_contiguous()
            and beta[0].is_contiguous() and gamma.stride(0) == beta.stride(0) and gamma.stride(0) % 4 == 0
            and gamma.data_ptr() % 16 == 0 and beta.data_ptr() % 16 == 0):
        return gamma.detach(), beta.detach(), gamma.stride(0)
    g = gamma.detach().float().contiguous()
    return g, beta.detach().float().contiguous(), g.shape[-1]


def _deterministic() -> bool:
    from ..utils import determinism
    return determinism.enabled()


class _GradStoreState:
    """First-touch weight gradients (fp32 ``tff`` path). ``record``: every weight-gradient GEMM notes the arena
    rows it writes (one tuple per call: weights and fused bias); ``store``: a call whose rows are all in ``rows``
    writes them with ``=`` instead of ``+=`` — the engine then zero-fills only the other columns of the gradient
    arena (:func:`first_touch_rows`, engine ``_tf_graph_step``)."""
    mode = None
    calls = None
    rows = frozenset()


_GS = _GradStoreState()

# gradient-completion listener (the data-parallel bucketer of ``distributed/cheetah.py``): called with the gradient-arena
# views a backward Function has finished writing — all of its kernels are enqueued on the current stream, so work
# enqueued after the call sees the final values
_READY = [None]


@contextlib.contextmanager
def grad_ready_listener(fn):
    prev = _READY[0]
    _READY[0] = fn
    try:
        yield
    finally:
        _READY[0] = prev


def client_sum(t: torch.Tensor, dim: int) -> torch.Tensor:
    """Σ over ``dim`` (> 0) of a client-stacked [C, ...] tensor. Deterministic mode: one reduction per client, so a
    client's bits never depend on how many clients share the launch (torch picks its reduction split from the
    whole tensor's shape) — R ranks × 1 replica then equal 1 rank × R replicas bit for bit."""
    if not _deterministic():
        return t.sum(dim)
    return torch.stack([t[c].sum(dim - 1) for c in range(t.shape[0])])


def _notify(views):
    if _READY[0] is not None and views:
        _READY[0](views)


@contextlib.contextmanager
def grad_store_record():
    """Record the weight-gradient rows written inside the block (yields the list of per-call tuples of
    (data_ptr, elements per client))."""
    prev = (_GS.mode, _GS.calls)
    _GS.mode, _GS.calls = "record", []
    try:
        yield _GS.calls
    finally:
        _GS.mode, _GS.calls = prev


@contextlib.contextmanager
def grad_store(rows):
    """Weight-gradient GEMMs whose rows (data_ptr) are all in ``rows`` store instead of accumulating."""
    prev = (_GS.mode, _GS.rows)
    _GS.mode, _GS.rows = "store", frozenset(rows)
    try:
        yield
    finally:
        _GS.mode, _GS.rows = prev


def first_touch_rows(calls):
    """(data_ptr set, [(data_ptr, elements per client)]) of the recorded calls whose rows no other recorded
    call writes — the rows a store-mode step may leave unzeroed."""
    count = {}
    for call in calls:
        for ptr, _ in call:
            count[ptr] = count.get(ptr, 0) + 1
    ok = [call for call in calls if all(count[ptr] == 1 for ptr, _ in call)]
    rows = [r for call in ok for r in call]
    return {ptr for ptr, _ in rows}, rows


class ResLink:
    """Hand-off of a residual-stream gradient between the two consumers of one activation, so autograd never
    has to add their two gradients in a separate pass (fp32 native path):

    * post-LN block (``x1 = LN(res = x, h = f(x))``): the LayerNorm's backward — which runs first — leaves dres
      in ``g`` and returns nothing for ``res``; the linear that reads ``x`` accumulates its data gradient into
      that buffer (``dx += dy·W`` in the GEMM epilogue) and returns it as the gradient of ``x``.
    * pre-LN block (``x' = x + f(LN(x))``, the add fused as ``res`` of the output linear): the output linear's
      backward leaves dres (= its incoming gradient) in ``g`` and returns nothing for ``res``; the LayerNorm that
      reads ``x`` adds it to its input gradient in the same kernel.

    Autograd runs the producer of the hand-off first in both patterns; should a consumer ever run first it
    ``closes`` the link, and the producer then returns its gradient the ordinary way (never lost)."""
    __slots__ = ("g", "closed")

    def __init__(self):
        self.g = None
        self.closed = False


class GeluLink:
    """Hand-off between a GELU'd linear (``gelu=True``, the producer: its pre-activation) and the linear that
    consumes its output: the consumer's data-gradient GEMM applies gelu'(pre) in its epilogue and the producer
    then skips its separate GELU-backward pass (fp32 native path). The consumer's backward runs first."""
    __slots__ = ("pre", "fused")

    def __init__(self):
        self.pre = None
        self.fused = False


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, res, gamma, beta, eps, p, seed, rpc, seed_dev, link=None, in_link=None):
        R, d = h.shape
        y = torch.empty_like(h)
        fused = res is not None or p > 0
        xsum = torch.empty_like(h) if fused else None
        mean = torch.empty(R, dtype=torch.float32, device=h.device)
        rstd = torch.empty(R, dtype=torch.float32, device=h.device)
        g, b, gcs = _client_rows(gamma, beta)
        name = "fa_ln_fwd" + _sfx(h)
        rc = _fn(name)(_p(h), _p(res), _c.c_int(R), _c.c_int(d), _c.c_int(rpc), _p(g), _p(b), _f(eps),
                       _c.c_uint32(_thr(p)), _f(1.0 / (1.0 - p) if p > 0 else 1.0), _c.c_uint32(seed & _M32),
                       _p(y), _p(xsum), _p(mean), _p(rstd), _p(seed_dev), _i64(gcs), _stream(h))
        _check(rc, name)
        ctx.save_for_backward(xsum if fused else h, mean, rstd, g)
        ctx.cfg = (p, seed, rpc, res is not None, fused, gamma.dtype, gcs)
        ctx.seed_dev = seed_dev
        ln16 = h.dtype in (torch.float32, torch.bfloat16)
        ctx.link = link if res is not None and ln16 else None    # post-LN: dres → link.g
        ctx.in_link = in_link if ln16 else None                  # pre-LN: dh += link.g
        # γ/β leaves with pre-assigned gradient-arena views: the backward kernel accumulates dγ/dβ into them
        ctx.own = (gamma, beta) if (gamma.is_leaf and beta.is_leaf and gamma.grad is not None and beta.grad is not None
                                    and gamma.grad.stride() == gamma.stride() and beta.grad.stride() == beta.stride()
                                    and gamma.grad.stride(0) == beta.grad.stride(0)) else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd, g = ctx.saved_tensors
        p, seed, rpc, has_res, fused, gdt, gcs = ctx.cfg
        seed_dev = ctx.seed_dev
        R, d = x.shape
        C = R // rpc
        dy = dy.to(x.dtype).contiguous()
        dres = torch.empty_like(x) if has_res else None
        dh = torch.empty_like(x)
        det = _deterministic()
        own = ctx.own is not None and not det
        if own:      # dγ/dβ atomically into the gradient arena rows (zeroed by the engine each step): no fill, no add
            dg, db = ctx.own[0].grad, ctx.own[1].grad
            dgcs = dg.stride(0)
        else:
            dg = torch.zeros(C, d, dtype=torch.float32, device=x.device)
            db = torch.zeros(C, d, dtype=torch.float32, device=x.device)
            dgcs = d
        name = "fa_ln_bwd" + _sfx(x)
        dadd = None
        if ctx.in_link is not None:
            if ctx.in_link.g is not None:
                dadd = ctx.in_link.g.reshape(R, d).to(x.dtype).contiguous()
                ctx.in_link.g = None
            else:
                ctx.in_link.closed = True
        if dadd is not None:
            name = "fa_ln_bwd_add" + _sfx(x)
            rc = _fn(name)(_p(dy), _p(x), _p(mean), _p(rstd), _c.c_int(C), _c.c_int(rpc), _c.c_int(d), _p(g),
                           _p(dres), _p(dh), _c.c_uint32(_thr(p)), _f(1.0 / (1.0 - p) if p > 0 else 1.0),
                           _c.c_uint32(seed & _M32), _p(dg), _p(db), _p(seed_dev), _i64(gcs), _i64(dgcs), _p(dadd),
                           _stream(x))
        else:
            rc = _fn(name)(_p(dy), _p(x), _p(mean), _p(rstd), _c.c_int(C), _c.c_int(rpc), _c.c_int(d), _p(g),
                           _p(dres), _p(dh), _c.c_uint32(_thr(p)), _f(1.0 / (1.0 - p) if p > 0 else 1.0),
                           _c.c_uint32(seed & _M32), _p(dg), _p(db), _p(seed_dev), _i64(gcs), _i64(dgcs), _stream(x))
        _check(rc, name)
        if ctx.link is not None and dres is not None and not ctx.link.closed:   # its other consumer adds into it
            ctx.link.g = dres
            dres = None
        if own:
            _notify([dg, db])
            return dh, dres, None, None, None, None, None, None, None, None, None
        if det:
            # the kernel's dgamma/dbeta reduce rows with fp32 atomics (arrival order → last bit): recompute them
            # as fixed-order column sums (deterministic-mode only; the kernel's dh/dres are atomic-free)
            xf, dyf = x.float().view(C, rpc, d), dy.float().view(C, rpc, d)
            xhat = (xf - mean.view(C, rpc, 1)) * rstd.view(C, rpc, 1)
            dg = client_sum(dyf * xhat, 1)
            db = client_sum(dyf, 1)
        return dh, dres, dg.to(gdt), db.to(gdt), None, None, None, None, None, None, None


def layer_norm(h: torch.Tensor, gamma: torch.Tensor, beta: torch.Tensor, eps: float, rows_per_client: int,
               res: torch.Tensor = None, p: float = 0.0, seed: int = 0, seed_dev: torch.Tensor = None,
               res_link: "ResLink" = None, in_link: "ResLink" = None) -> torch.Tensor:
    """LN(res + dropout_p(h)) over the last dim of 2-D ``h`` [R, d]; gamma/beta ``[C, d]``.
    ``seed_dev`` (GPU): a [1] uint32/int32 device step counter — the kernels then use
    seed + counter·1000003, so a captured HIP graph draws new dropout masks on every replay.
    ``res_link`` / ``in_link``: :class:`ResLink` hand-offs of the residual-stream gradient (fp32 native path)."""
    assert h.dim() == 2 and h.shape[0] % rows_per_client == 0
    if use_native(h):
        _sfx(h)
        assert h.is_contiguous() and (res is None or (res.is_contiguous() and res.dtype == h.dtype))
        return _LayerNorm.apply(h, res, gamma, beta, float(eps), float(p), int(seed), int(rows_per_client), seed_dev,
                                res_link, in_link)
    return _ln_ref(h, res, gamma, beta, eps, p, seed, rows_per_client)


# ----------------------------------------------------------------------------------------- GELU
class _Gelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        y = torch.empty_like(x)
        name = "fa_gelu_fwd" + _sfx(x)
        _check(_fn(name)(_p(x), _p(y), _i64(x.numel()), _stream(x)), name)
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        gy = gy.to(x.dtype).contiguous()
        gx = torch.empty_like(x)
        name = "fa_gelu_bwd" + _sfx(x)
        _check(_fn(name)(_p(x), _p(gy), _p(gx), _i64(x.numel()), _stream(x)), name)
        return gx


def gelu(x: torch.Tensor) -> torch.Tensor:
    if use_native(x):
        assert x.is_contiguous() and x.numel() % (8 if _sfx(x) == "" else 4) == 0
        return _Gelu.apply(x)
    return torch.nn.functional.gelu(x.float()).to(x.dtype)


# ------------------------------------------------------------------------------------ attention
def _attn_ref(q, k, v, kmask, S, H, p, seed):
    T, dm = q.shape
    CB = T // S
    ct = _ct(q)
    qh = q.to(ct).view(CB, S, H, 64).transpose(1, 2)
    kh = k.to(ct).view(CB, S, H, 64).transpose(1, 2)
    vh = v.to(ct).view(CB, S, H, 64).transpose(1, 2)
    s = qh @ kh.transpose(-1, -2) / math.sqrt(64.0)
    if kmask is not None:
        s = s.masked_fill(~kmask.view(CB, 1, 1, S).bool(), float("-inf"))
    pr = torch.softmax(s, -1).nan_to_num(0.0)
    if p > 0:
        bh = torch.arange(CB * H, device=q.device).view(CB, H, 1, 1)
        qi = torch.arange(S, device=q.device).view(1, 1, S, 1)
        ki = torch.arange(S, device=q.device).view(1, 1, 1, S)
        keep = dropout_keep(seed, bh * 65536 + qi, ki, p)
        pr = torch.where(keep, pr / (1.0 - p), torch.zeros_like(pr))
    o = (pr @ vh).transpose(1, 2).reshape(T, dm)
    return o.to(q.dtype)


class _Attention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, kmask, S, H, p, seed, seed_dev):
        T, dm = q.shape
        CB = T // S
        o = torch.empty(T, dm, dtype=q.dtype, device=q.device)
        lse = torch.empty(CB, H, S, dtype=torch.float32, device=q.device)
        scale = 1.0 / math.sqrt(64.0)
        name = "fa_attn_fwd" + _sfx(q)
        rc = _fn(name)(_p(q), _c.c_int(q.stride(0)), _p(k), _c.c_int(k.stride(0)), _p(v),
                       _c.c_int(v.stride(0)), _p(o), _c.c_int(dm), _p(kmask), _p(lse), _c.c_int(CB),
                       _c.c_int(S), _c.c_int(H), _f(scale), _c.c_uint32(_thr(p)),
                       _f(1.0 / (1.0 - p) if p > 0 else 1.0), _c.c_uint32(seed & _M32), _p(seed_dev),
                       _stream(q))
        _check(rc, name)
        ctx.save_for_backward(q, k, v, o, lse, kmask)
        ctx.cfg = (S, H, p, seed)
        ctx.seed_dev = seed_dev
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, kmask = ctx.saved_tensors
        S, H, p, seed = ctx.cfg
        T, dm = q.shape
        CB = T // S
        do = do.to(q.dtype).contiguous()
        dq = torch.empty(T, dm, dtype=q.dtype, device=q.device)
        dk = torch.empty_like(dq)
        dv = torch.empty_like(dq)
        D = torch.empty(CB, H, S, dtype=torch.float32, device=q.device)
        name = "fa_attn_bwd" + _sfx(q)
        rc = _fn(name)(_p(q), _c.c_int(q.stride(0)), _p(k), _c.c_int(k.stride(0)), _p(v),
                       _c.c_int(v.stride(0)), _p(o), _c.c_int(dm), _p(do), _c.c_int(dm), _p(kmask), _p(lse),
                       _p(D), _p(dq), _c.c_int(dm), _p(dk), _c.c_int(dm), _p(dv), _c.c_int(dm),
                       _c.c_int(CB), _c.c_int(S), _c.c_int(H), _f(1.0 / math.sqrt(64.0)),
                       _c.c_uint32(_thr(p)), _f(1.0 / (1.0 - p) if p > 0 else 1.0),
                       _c.c_uint32(seed & _M32), _p(ctx.seed_dev), _stream(q))
        _check(rc, name)
        return dq, dk, dv, None, None, None, None, None, None


class _AttentionQKV(torch.autograd.Function):
    """Attention over the fused q/k/v projection output ``qkv`` [T, 3·dm] taken whole: the backward kernels write
    dq / dk / dv straight into the column slices of ONE gradient buffer — three separate slice gradients would
    make autograd zero a [T, 3·dm] buffer and copy each slice into it."""

    @staticmethod
    def forward(ctx, qkv, kmask, S, H, p, seed, seed_dev):
        dm = qkv.shape[1] // 3
        q, k, v = qkv[:, :dm], qkv[:, dm:2 * dm], qkv[:, 2 * dm:]
        o = _Attention.forward(ctx, q, k, v, kmask, S, H, p, seed, seed_dev)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse, kmask = ctx.saved_tensors
        S, H, p, seed = ctx.cfg
        T, dm = q.shape
        CB = T // S
        do = do.to(q.dtype).contiguous()
        dqkv = torch.empty(T, 3 * dm, dtype=q.dtype, device=q.device)
        D = torch.empty(CB, H, S, dtype=torch.float32, device=q.device)
        ld = 3 * dm
        name = "fa_attn_bwd" + _sfx(q)
        rc = _fn(name)(_p(q), _c.c_int(q.stride(0)), _p(k), _c.c_int(k.stride(0)), _p(v),
                       _c.c_int(v.stride(0)), _p(o), _c.c_int(dm), _p(do), _c.c_int(dm), _p(kmask), _p(lse),
                       _p(D), _p(dqkv), _c.c_int(ld), _p(dqkv[:, dm:]), _c.c_int(ld), _p(dqkv[:, 2 * dm:]),
                       _c.c_int(ld), _c.c_int(CB), _c.c_int(S), _c.c_int(H), _f(1.0 / math.sqrt(64.0)),
                       _c.c_uint32(_thr(p)), _f(1.0 / (1.0 - p) if p > 0 else 1.0),
                       _c.c_uint32(seed & _M32), _p(ctx.seed_dev), _stream(q))
        _check(rc, name)
        return dqkv, None, None, None, None, None, None


def attention_qkv(qkv, S: int, H: int, kmask: torch.Tensor = None, p: float = 0.0, seed: int = 0,
                  seed_dev: torch.Tensor = None):
    """:func:`attention` over the fused projection output ``qkv`` [CB·S, 3·H·64] (q | k | v column blocks)."""
    dm = qkv.shape[1] // 3
    if use_native(qkv) and qkv.is_contiguous():
        vec = 8 if _sfx(qkv) == "" else 4
        assert S <= 256 and dm == H * 64 and qkv.shape[0] % S == 0 and (3 * dm) % vec == 0
        km = None if kmask is None else kmask.to(torch.uint8).contiguous()
        return _AttentionQKV.apply(qkv, km, int(S), int(H), float(p), int(seed), seed_dev)
    return attention(qkv[:, :dm], qkv[:, dm:2 * dm], qkv[:, 2 * dm:], S, H, kmask=kmask, p=p, seed=seed,
                     seed_dev=seed_dev)


def attention(q, k, v, S: int, H: int, kmask: torch.Tensor = None, p: float = 0.0, seed: int = 0,
              seed_dev: torch.Tensor = None):
    """Multi-head self-attention over token-major ``[CB·S, H·64]`` q/k/v (row stride may exceed
    H·64, e.g. column slices of a fused QKV output); ``kmask`` [CB, S] (nonzero = attend);
    ``seed_dev`` as in :func:`layer_norm`."""
    assert q.dim() == 2 and q.shape[1] == H * 64 and q.shape[0] % S == 0
    if use_native(q):
        vec = 8 if _sfx(q) == "" else 4
        assert S <= 256
        for t in (q, k, v):
            assert t.dtype == q.dtype and t.stride(1) == 1 and t.stride(0) % vec == 0
        km = None if kmask is None else kmask.to(torch.uint8).contiguous()
        return _Attention.apply(q, k, v, km, int(S), int(H), float(p), int(seed), seed_dev)
    return _attn_ref(q, k, v, kmask, S, H, p, seed)


# ------------------------------------------------------------------------ client-batched linear
def _segments(views):
    """(base, client stride, per-segment element offsets, row boundaries) of [C, n_i, ...] arena
    views (fp32, or the bf16 shadow) sharing one client stride (the q/k/v slots of a fused projection)."""
    base = views[0]
    cs = base.stride(0)
    es = base.element_size()
    off, lo = [], [0]
    for v in views:
        assert v.dtype == base.dtype and v.stride(0) == cs, "segments must share dtype and client stride"
        assert v.stride(-1) == 1 and (v.dim() < 3 or v.stride(1) == v.shape[2]), "segment rows must be contiguous"
        off.append((v.data_ptr() - base.data_ptr()) // es)
        lo.append(lo[-1] + v.shape[1])
    return base, cs, (_c.c_int64 * 4)(*(off + [0] * (4 - len(off)))), (_c.c_int * 5)(*(lo + [0] * (5 - len(lo))))


def native_linear_ok(M: int, N: int, K: int, nseg: int = 1, dtype=torch.bfloat16) -> bool:
    """Shapes the batched-GEMM kernels take: bf16 needs 16-byte vectors along every contiguous dim;
    the fp32 kernels take any shape (an element-wise staging variant covers unaligned ones)."""
    if dtype == torch.float32:
        return 1 <= nseg <= 4 and M > 0 and N > 0 and K > 0
    return K % 8 == 0 and N % 8 == 0 and 1 <= nseg <= 4 and M > 0


class _ClientLinear(torch.autograd.Function):
    """y[c] = act(x[c] · W[c]ᵀ + b[c]) with W, b read straight from the fp32 client arena (one or
    several slots), bf16 activations; backward adds dW / db straight into the gradient arena
    (the leaves' pre-assigned ``.grad`` views) — no dense per-step weight copies either way."""

    @staticmethod
    def forward(ctx, x, gelu, n_w, shadows, res, links, *params):
        ws, bs = params[:n_w], params[n_w:]
        # links = (dx_link, res_link, gelu_out, gelu_in): ResLink / GeluLink | None each (fp32 / bf16 native kernels)
        dl, rl, go, gi = links if links is not None else (None, None, None, None)
        ctx.dx_link, ctx.res_link = (dl, rl) if x.dtype in (torch.float32, torch.bfloat16) else (None, None)
        ctx.gelu_out, ctx.gelu_in = (go, gi) if x.dtype in (torch.float32, torch.bfloat16) else (None, None)
        C, M, K = x.shape
        N = sum(w.shape[1] for w in ws)
        # bf16 shadow of the weights (refreshed once per step by the engine) when given: half the
        # B-operand bytes and no per-tile fp32→bf16 conversion; otherwise the fp32 arena itself
        wsrc = shadows if shadows else ws
        wb, wcs, woff, lo = _segments(wsrc)
        wh = 1 if wsrc[0].dtype == torch.bfloat16 else 0
        if bs:
            bb, bcs, boff, blo = _segments(bs)
            assert list(blo) == list(lo)
        else:
            bb, bcs, boff = None, 0, None
        y = torch.empty(C, M, N, dtype=x.dtype, device=x.device)
        y2 = torch.empty_like(y) if gelu else None
        fused_res = res is not None and x.dtype == torch.float32 and not gelu
        fused_res16 = (res is not None and x.dtype == torch.bfloat16 and not gelu and res.dtype == torch.bfloat16
                       and res.shape == (C, M, N) and res.is_contiguous())
        if fused_res16:                 # bf16: the same residual epilogue
            rc = _fn("fa_bgemm_fwd_res")(_p(x), _i64(M * K), _c.c_int(K), _p(wb), _c.c_int(wh), _i64(wcs), woff, _p(bb),
                                         _i64(bcs), boff, lo, _c.c_int(len(ws)), _p(y), _i64(M * N), _c.c_int(N),
                                         None, _p(res), _c.c_int(C), _c.c_int(M), _c.c_int(N), _c.c_int(K), _stream(x))
            fused_res = True
        elif fused_res:                 # y = x·Wᵀ + b + res in the GEMM epilogue (pre-LN residual stream)
            assert wh == 0 and res.shape == (C, M, N) and res.dtype == torch.float32 and res.is_contiguous()
            rc = _fn("fa_bgemm_fwd_res_f32")(_p(x), _i64(M * K), _c.c_int(K), _p(wb), _i64(wcs), woff, _p(bb),
                                             _i64(bcs), boff, lo, _c.c_int(len(ws)), _p(y), _i64(M * N), _c.c_int(N),
                                             _p(res), _i64(M * N), _c.c_int(N), _c.c_int(C), _c.c_int(M),
                                             _c.c_int(N), _c.c_int(K), _stream(x))
        elif x.dtype == torch.float32:    # fp32 activations: the fp32 kernels read the fp32 arena
            assert wh == 0
            rc = _fn("fa_bgemm_fwd_f32")(_p(x), _i64(M * K), _c.c_int(K), _p(wb), _i64(wcs), woff, _p(bb),
                                         _i64(bcs), boff, lo, _c.c_int(len(ws)), _p(y), _i64(M * N), _c.c_int(N),
                                         _p(y2), _c.c_int(C), _c.c_int(M), _c.c_int(N), _c.c_int(K), _stream(x))
        else:
            rc = _fn("fa_bgemm_fwd")(_p(x), _i64(M * K), _c.c_int(K), _p(wb), _c.c_int(wh), _i64(wcs), woff, _p(bb),
                                     _i64(bcs), boff,
                                     lo, _c.c_int(len(ws)), _p(y), _i64(M * N), _c.c_int(N), _p(y2), _c.c_int(C),
                                     _c.c_int(M), _c.c_int(N), _c.c_int(K), _stream(x))
        _check(rc, "fa_bgemm_fwd" + _sfx(x))
        if res is not None and not fused_res:
            y = y + res.to(y.dtype)
        ctx.save_for_backward(x, y if gelu else None)
        ctx.ws, ctx.bs, ctx.gelu, ctx.wsrc = ws, bs, gelu, wsrc
        ctx.has_res = res is not None
        if gelu and ctx.gelu_out is not None:
            ctx.gelu_out.pre = y            # the consumer's dgrad applies gelu'(pre)
        return y2 if gelu else y

    @staticmethod
    def backward(ctx, g):
        x, pre = ctx.saved_tensors
        ws, bs = ctx.ws, ctx.bs
        C, M, K = x.shape
        N = sum(w.shape[1] for w in ws)
        g_res = g if ctx.has_res and ctx.needs_input_grad[4] else None   # y = … + res: dres = dy
        if g_res is not None and ctx.res_link is not None and not ctx.res_link.closed:   # the LN adds it to its dh
            ctx.res_link.g = g_res
            g_res = None
        g = g.to(x.dtype).contiguous()
        sfx = _sfx(x)
        if ctx.gelu and ctx.gelu_out is not None and ctx.gelu_out.fused:
            ctx.gelu_out.pre = None         # g is already the gradient through the GELU
        elif ctx.gelu:
            gp = torch.empty_like(pre)
            _check(_fn("fa_gelu_bwd" + sfx)(_p(pre), _p(g), _p(gp), _i64(pre.numel()), _stream(pre)),
                   "fa_gelu_bwd" + sfx)
            g = gp
        dx = None
        if ctx.needs_input_grad[0]:
            wb, wcs, woff, lo = _segments(ctx.wsrc)
            wh = 1 if ctx.wsrc[0].dtype == torch.bfloat16 else 0
            link = ctx.dx_link
            acc = link is not None and link.g is not None and link.g.dtype == x.dtype and link.g.is_contiguous()
            if link is not None and not acc:
                link.closed = True
            gl = ctx.gelu_in
            dgelu = not acc and gl is not None and gl.pre is not None and gl.pre.shape == x.shape and \
                gl.pre.dtype == x.dtype and gl.pre.is_contiguous()
            if dgelu and not sfx:   # bf16: the same GELU backward in the dgrad epilogue
                dx = torch.empty_like(x)
                rc = _fn("fa_bgemm_dgrad_dgelu")(_p(g), _i64(M * N), _c.c_int(N), _p(wb), _c.c_int(wh), _i64(wcs),
                                                 woff, lo, _c.c_int(len(ws)), _p(dx), _i64(M * K), _c.c_int(K),
                                                 _p(gl.pre), _c.c_int(C), _c.c_int(M), _c.c_int(N), _c.c_int(K),
                                                 _stream(x))
                gl.fused = True
                gl.pre = None
            elif dgelu:   # x = gelu(pre) of the previous linear: return the gradient w.r.t. pre directly
                dx = torch.empty_like(x)
                rc = _fn("fa_bgemm_dgrad_dgelu_f32")(_p(g), _i64(M * N), _c.c_int(N), _p(wb), _i64(wcs), woff, lo,
                                                     _c.c_int(len(ws)), _p(dx), _i64(M * K), _c.c_int(K),
                                                     _p(gl.pre), _c.c_int(C), _c.c_int(M), _c.c_int(N), _c.c_int(K),
                                                     _stream(x))
                gl.fused = True
                gl.pre = None
            elif acc and not sfx:   # bf16: dx = dy·W + (the other consumer's gradient), in the epilogue, in place
                dx = link.g.view(C, M, K)
                link.g = None
                rc = _fn("fa_bgemm_dgrad_add")(_p(g), _i64(M * N), _c.c_int(N), _p(wb), _c.c_int(wh), _i64(wcs), woff,
                                               lo, _c.c_int(len(ws)), _p(dx), _i64(M * K), _c.c_int(K), _p(dx),
                                               _c.c_int(C), _c.c_int(M), _c.c_int(N), _c.c_int(K), _stream(x))
            elif acc:   # x's other consumer (a post-LN residual) left its gradient: add ours into it
                dx = link.g.view(C, M, K)
                link.g = None
                assert dx.dtype == torch.float32 and dx.is_contiguous()
                rc = _fn("fa_bgemm_dgrad_acc_f32")(_p(g), _i64(M * N), _c.c_int(N), _p(wb), _i64(wcs), woff, lo,
                                                   _c.c_int(len(ws)), _p(dx), _i64(M * K), _c.c_int(K), _c.c_int(C),
                                                   _c.c_int(M), _c.c_int(N), _c.c_int(K), _stream(x))
            elif sfx:
                dx = torch.empty_like(x)
                rc = _fn("fa_bgemm_dgrad_f32")(_p(g), _i64(M * N), _c.c_int(N), _p(wb), _i64(wcs), woff, lo,
                                               _c.c_int(len(ws)), _p(dx), _i64(M * K), _c.c_int(K), _c.c_int(C),
                                               _c.c_int(M), _c.c_int(N), _c.c_int(K), _stream(x))
            else:
                dx = torch.empty_like(x)
                rc = _fn("fa_bgemm_dgrad")(_p(g), _i64(M * N), _c.c_int(N), _p(wb), _c.c_int(wh), _i64(wcs), woff, lo,
                                           _c.c_int(len(ws)), _p(dx), _i64(M * K), _c.c_int(K), _c.c_int(C),
                                           _c.c_int(M), _c.c_int(N), _c.c_int(K), _stream(x))
            _check(rc, "fa_bgemm_dgrad" + sfx)
            if not acc and link is not None and link.g is not None:   # (not reached: links are fp32-only)
                dx = dx + link.g.view(C, M, K).to(dx.dtype)
                link.g = None
        # weight gradients: into the arena views when the engine pre-assigned them, else returned
        own = all(w.is_leaf and w.grad is not None for w in ws)
        if own:
            gviews = [w.grad for w in ws]
            out_w = [None] * len(ws)
        else:
            dense = torch.zeros(C, N, K, dtype=torch.float32, device=x.device)
            gviews, out_w, r = [], [], 0
            for w in ws:
                v = dense[:, r:r + w.shape[1]]
                gviews.append(v)
                out_w.append(v.view_as(w))
                r += w.shape[1]
        gb, gcs, goff, glo = _segments(gviews)
        # fp32, engine-owned bias slots, not deterministic: the bias gradient comes out of the weight-gradient GEMM's
        # own reads of g (one pass instead of a separate column reduction)
        fused_b = (bool(bs) and all(b.is_leaf and b.grad is not None for b in bs) and not _deterministic())
        rows_w = [(v.data_ptr(), v[0].numel()) for v in gviews] if own else []
        rows_b = [(b.grad.data_ptr(), b.grad[0].numel()) for b in bs] if fused_b else []

        def first_touch(rows):   # store mode: these rows are written by this call only (not zero-filled)
            return int(_GS.mode == "store" and bool(rows) and all(ptr in _GS.rows for ptr, _ in rows))
        rc = -1
        if fused_b:
            bb_, bcs_, boff_, blo_ = _segments([b.grad for b in bs])
            if list(blo_) == list(glo):
                rc = _fn("fa_bgemm_wgrad_bias" + sfx)(_p(g), _i64(M * N), _c.c_int(N), _p(x), _i64(M * K), _c.c_int(K),
                                                   _p(gb), _i64(gcs), goff, glo, _c.c_int(len(ws)), _p(bb_),
                                                   _i64(bcs_), boff_, _c.c_int(C), _c.c_int(M), _c.c_int(N),
                                                   _c.c_int(K), _c.c_int(first_touch(rows_w + rows_b)), _stream(x))
            fused_b = rc == 0
        if fused_b:
            if _GS.mode == "record":
                _GS.calls.append(tuple(rows_w + rows_b))
        elif sfx:
            rc = _fn("fa_bgemm_wgrad_st_f32")(_p(g), _i64(M * N), _c.c_int(N), _p(x), _i64(M * K), _c.c_int(K),
                                              _p(gb), _i64(gcs), goff, glo, _c.c_int(len(ws)), _c.c_int(C),
                                              _c.c_int(M), _c.c_int(N), _c.c_int(K), _c.c_int(first_touch(rows_w)),
                                              _stream(x))
            if _GS.mode == "record" and rows_w:
                _GS.calls.append(tuple(rows_w))
        else:
            rc = _fn("fa_bgemm_wgrad_bias")(_p(g), _i64(M * N), _c.c_int(N), _p(x), _i64(M * K), _c.c_int(K), _p(gb),
                                            _i64(gcs), goff, glo, _c.c_int(len(ws)), None, _i64(0), None,
                                            _c.c_int(C), _c.c_int(M), _c.c_int(N), _c.c_int(K),
                                            _c.c_int(first_touch(rows_w)), _stream(x))
            if _GS.mode == "record" and rows_w:
                _GS.calls.append(tuple(rows_w))
        _check(rc, "fa_bgemm_wgrad" + sfx)
        out_b = []
        if bs and fused_b:
            out_b = [None] * len(bs)
        elif bs:
            # column sums of g straight into the gradient arena (or a dense [C, N] when not owned)
            own_b = all(b.is_leaf and b.grad is not None for b in bs)
            if own_b:
                bviews = [b.grad for b in bs]
                out_b = [None] * len(bs)
            else:
                dense_b = torch.zeros(C, N, dtype=torch.float32, device=x.device)
                bviews, r = [], 0
                for b in bs:
                    bviews.append(dense_b[:, r:r + b.shape[1]])
                    out_b.append(dense_b[:, r:r + b.shape[1]])
                    r += b.shape[1]
            if _deterministic():
                # fixed-order column sums instead of the kernel's fp32 atomics (deterministic mode)
                gs = client_sum(g.view(C, M, N).float(), 1)
                r = 0
                for bv in bviews:
                    bv.add_(gs[:, r:r + bv.shape[1]])
                    r += bv.shape[1]
                if own:
                    _notify(list(gviews) + list(bviews))
                return (dx, None, None, None, g_res, None, *out_w, *out_b)
            bb, bcs, boff, blo = _segments(bviews)
            rc = _fn("fa_bias_grad" + sfx)(_p(g), _i64(M * N), _c.c_int(N), _p(bb), _i64(bcs), boff, blo,
                                     _c.c_int(len(bs)), _c.c_int(C), _c.c_int(M), _c.c_int(N), _stream(x))
            _check(rc, "fa_bias_grad" + sfx)
        if own:
            done = list(gviews)
            if bs and (fused_b or all(b.is_leaf and b.grad is not None for b in bs)):
                done += [b.grad for b in bs]
            _notify(done)
        return (dx, None, None, None, g_res, None, *out_w, *out_b)


def client_linear(x: torch.Tensor, weights, biases=None, gelu: bool = False, shadows=None,
                  res: torch.Tensor = None, dx_link: "ResLink" = None, res_link: "ResLink" = None,
                  gelu_out: "GeluLink" = None, gelu_in: "GeluLink" = None) -> torch.Tensor:
    """Per-client linear over client-stacked activations ``x`` [C, M, K]: ``weights`` is a list of
    [C, n_i, K] fp32 arena views (concatenated along the output dim), ``biases`` the matching
    [C, n_i] views or None; ``gelu`` fuses the exact-erf GELU into the epilogue. ``shadows``: the
    same slots of a bf16 copy of the arena (current for this step) — the GEMMs then read bf16
    weights; gradients always land in the fp32 arena. CUDA → the batched MFMA GEMM kernels at the
    activation dtype (bf16, or fp32 through ``tf_f32_kernels.hip``); CPU → the fp32 PyTorch reference.
    ``res`` [C, M, N] (no GELU): the result is ``res + linear(x)`` — at fp32 added in the GEMM epilogue (the residual
    stream of a pre-LN block without a separate add pass). ``dx_link`` / ``res_link``: :class:`ResLink`
    hand-offs of the residual-stream gradient; ``gelu_out`` (on a ``gelu=True`` linear) / ``gelu_in`` (on the
    linear reading its output): :class:`GeluLink`, the GELU backward folded into the consumer's dgrad GEMM."""
    assert res is None or not gelu
    weights = list(weights)
    biases = list(biases) if biases else []
    C, M, K = x.shape
    N = sum(w.shape[1] for w in weights)
    if use_native(x) and native_linear_ok(M, N, K, len(weights), x.dtype):
        _sfx(x)
        sh = tuple(shadows) if shadows and x.dtype == torch.bfloat16 else None
        if sh is not None:
            assert len(sh) == len(weights) and all(t.shape == w.shape for t, w in zip(sh, weights))
        r = res.contiguous() if res is not None else None
        links = (dx_link, res_link, gelu_out, gelu_in) \
            if any(t is not None for t in (dx_link, res_link, gelu_out, gelu_in)) else None
        return _ClientLinear.apply(x.contiguous(), bool(gelu), len(weights), sh, r, links, *weights, *biases)
    w = torch.cat([t.reshape(C, t.shape[1], K) for t in weights], 1)
    y = torch.bmm(x.float(), w.float().transpose(1, 2))
    if biases:
        y = y + torch.cat(list(biases), 1).float().unsqueeze(1)
    if gelu:
        y = torch.nn.functional.gelu(y.to(x.dtype).float())
    y = y.to(x.dtype)
    return y if res is None else res + y
