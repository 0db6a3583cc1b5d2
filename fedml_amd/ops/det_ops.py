"""Deterministic accumulation for the native kernels (csrc/detacc.h, csrc/det_kernels.hip).

The conv / BN / LayerNorm / bias-gradient kernels reduce across workgroups with fp32 global atomics, whose
result depends on arrival order. ``DetAccumulator`` registers up to 16 fp32 device tensors: while
it is active, every atomic into them goes to a 128-bit fixed-point shadow instead (integer adds are
associative → the same bits in any order), and ``flush(t)`` rounds the shadow of ``t`` into ``t`` (+=) and
clears it. Kernel code does not change between the modes; the registry is process-global (one device
table per kernel translation unit), so one accumulator is active at a time.

Used by ``NativeResNetStep`` in deterministic mode (utils/determinism.py); the reference's counterpart
is ``torch.backends.cudnn.deterministic = True`` in its seeding path (``fedml/__init__.py:51``), which
keeps cuDNN on order-fixed reductions."""
import ctypes

import torch

from .fl_ops import _check, _fn, _i64, _p, _stream

MAXR = 16
# deterministic mode plans every client-batched work split for this many clients (csrc/common.h fa_plan_c)
PLAN_CLIENTS = 64
_TUS = ("det", "bn", "conv", "conv1x1", "conv3x3", "wgrad", "transformer", "tf_f32", "bgemm")
_active = [None]


def active():
    return _active[0]


def set_plan_clients(n: int):
    """Plan the native kernels' work splits for ``n`` clients whatever a launch's C is (0: the launch's C)."""
    _check(_fn("fa_set_plan_clients")(ctypes.c_int(int(n))), "fa_set_plan_clients")


class _Table(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("lo", ctypes.c_void_p * MAXR), ("len", ctypes.c_int64 * MAXR),
                ("acc", ctypes.c_void_p * MAXR), ("bad", ctypes.c_void_p)]


def _set_all(tab: _Table):
    torch.cuda.synchronize()     # no kernel of another stream may be mid-flight while the tables change
    for tu in _TUS:
        _check(_fn(f"fa_det_set_{tu}")(ctypes.byref(tab)), f"fa_det_set_{tu}")


class DetAccumulator:
    """Targets are registered eagerly (never while a stream captures): the device tables are set with a
    synchronous copy. Shadows persist for the accumulator's lifetime, so captured flush launches stay
    valid when more targets are added later (e.g. the buffers of another batch geometry)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.targets, self.acc = [], []
        self.bad = torch.zeros(1, dtype=torch.int32, device=self.device)

    def _table(self) -> _Table:
        tab = _Table()
        tab.n = len(self.targets)
        for i, (t, a) in enumerate(zip(self.targets, self.acc)):
            tab.lo[i] = t.data_ptr()
            tab.len[i] = t.numel()
            tab.acc[i] = a.data_ptr()
        tab.bad = self.bad.data_ptr()
        return tab

    def register(self, t):
        if t is None:
            return
        if any(u.data_ptr() == t.data_ptr() and u.numel() == t.numel() for u in self.targets):
            return
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("deterministic targets are contiguous fp32 device tensors")
        if len(self.targets) >= MAXR:
            raise ValueError(f"at most {MAXR} deterministic targets")
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("register deterministic targets before graph capture")
        self.targets.append(t)
        self.acc.append(torch.zeros(2 * t.numel(), dtype=torch.int64, device=t.device))
        if _active[0] is self:
            _set_all(self._table())

    def activate(self):
        if _active[0] is self:
            return
        if _active[0] is not None:
            raise RuntimeError("another deterministic accumulator is active (close it first)")
        _set_all(self._table())
        _active[0] = self

    def close(self):
        if _active[0] is self:
            _set_all(_Table())
            _active[0] = None

    def _find(self, t):
        p, n = t.data_ptr(), t.numel()
        for base, a in zip(self.targets, self.acc):
            d = p - base.data_ptr()
            if d >= 0 and d % 4 == 0 and d // 4 + n <= base.numel():
                return a, d // 4
        raise KeyError("tensor is not inside a registered deterministic target")

    def flush(self, t):
        """t (a registered target or a contiguous slice of one) += its accumulated sums; clears them."""
        a, off = self._find(t)
        rc = _fn("fa_det_flush")(_p(t), ctypes.c_void_p(a.data_ptr() + 16 * off), _i64(t.numel()), _p(self.bad),
                                 _stream(t))
        _check(rc, "fa_det_flush")

    def poisoned(self) -> bool:
        return bool(int(self.bad.item()))
