"""Flat parameter arena.

Every model is described by a ``ParamLayout``: the ordered state_dict keys with
(offset, shape, dtype), each tensor starting on a 256-byte boundary (offsets
computed by the native runtime, ``fr_layout``). The global model is one fp32
vector [P]; a client stack is [C, P]; optimizer state, error-feedback residuals
and aggregation accumulators share the same layout. state_dict conversion
happens only at API edges (``get_model_params``, checkpoints, user trainers) —
aggregation, compression and communication move the flat buffers
(one RCCL collective / one kernel instead of per-key Python loops,
`simulation/single_process/fedavg/fedavg_api.py:206-221`).
"""
import ctypes
from collections import OrderedDict
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional

import numpy as np
import torch

from ..utils.native_runtime import runtime_lib

ALIGN_BYTES = 256


@dataclass
class Slot:
    key: str
    offset: int
    numel: int
    shape: tuple
    dtype: torch.dtype
    is_weight: bool   # False for BN running stats / counters (excluded from robust norms)
    trainable: bool


def is_weight_param(k: str) -> bool:
    """Reference `core/robustness/robust_aggregation.py:35-40`."""
    return "running_mean" not in k and "running_var" not in k and "num_batches_tracked" not in k


class ParamLayout:
    def __init__(self, state_dict: Dict[str, torch.Tensor], trainable_keys: Optional[Iterable[str]] = None,
                 align_bytes: int = ALIGN_BYTES):
        keys = list(state_dict.keys())
        numels = np.array([max(1, state_dict[k].numel()) for k in keys], dtype=np.int64)
        offsets = np.zeros(len(keys), dtype=np.int64)
        lib = runtime_lib()
        if lib is not None and len(keys):
            total = lib.fr_layout(len(keys), numels.ctypes.data_as(ctypes.c_void_p), 4, align_bytes,
                                  offsets.ctypes.data_as(ctypes.c_void_p))
        else:
            a = align_bytes // 4
            off = 0
            for i, n in enumerate(numels):
                off = (off + a - 1) // a * a
                offsets[i] = off
                off += int(n)
            total = (off + a - 1) // a * a
        tk = set(trainable_keys) if trainable_keys is not None else None
        self.slots: List[Slot] = []
        for k, off, n in zip(keys, offsets, numels):
            t = state_dict[k]
            self.slots.append(Slot(k, int(off), int(t.numel()), tuple(t.shape), t.dtype, is_weight_param(k),
                                   (tk is None and t.is_floating_point()) or (tk is not None and k in tk)))
        self.size = int(total)
        self._by_key = {s.key: s for s in self.slots}

    @classmethod
    def from_module(cls, module: torch.nn.Module) -> "ParamLayout":
        sd = module.state_dict()
        trainable = {n for n, p in module.named_parameters() if p.requires_grad}
        return cls(sd, trainable)

    def __len__(self):
        return len(self.slots)

    def keys(self):
        return [s.key for s in self.slots]

    def slot(self, key) -> Slot:
        return self._by_key[key]

    # ---- conversion -------------------------------------------------------------------
    def flatten(self, state_dict: Dict[str, torch.Tensor], out: Optional[torch.Tensor] = None,
                device=None) -> torch.Tensor:
        if out is None:
            dev = device if device is not None else next(iter(state_dict.values())).device
            out = torch.zeros(self.size, dtype=torch.float32, device=dev)
        for s in self.slots:
            out[s.offset:s.offset + s.numel].copy_(state_dict[s.key].reshape(-1).to(torch.float32), non_blocking=True)
        return out

    def unflatten(self, flat: torch.Tensor, device=None, clone: bool = True) -> "OrderedDict[str, torch.Tensor]":
        sd = OrderedDict()
        for s in self.slots:
            v = flat[s.offset:s.offset + s.numel].view(s.shape)
            if s.dtype.is_floating_point:
                v = v.to(s.dtype)
                if clone and v.data_ptr() == flat.data_ptr() + s.offset * flat.element_size():
                    v = v.clone()
            else:
                v = torch.round(v).to(s.dtype)
            sd[s.key] = v if device is None else v.to(device)
        return sd

    def views(self, flat: torch.Tensor) -> "OrderedDict[str, torch.Tensor]":
        """Zero-copy fp32 views into a flat buffer (for in-place kernels)."""
        return OrderedDict((s.key, flat[..., s.offset:s.offset + s.numel].view(*flat.shape[:-1], *s.shape))
                           for s in self.slots)

    def weight_mask(self, device=None) -> torch.Tensor:
        m = torch.zeros(self.size, dtype=torch.uint8, device=device)
        for s in self.slots:
            if s.is_weight:
                m[s.offset:s.offset + s.numel] = 1
        return m

    def trainable_mask(self, device=None) -> torch.Tensor:
        m = torch.zeros(self.size, dtype=torch.uint8, device=device)
        for s in self.slots:
            if s.trainable:
                m[s.offset:s.offset + s.numel] = 1
        return m

    def alloc_stack(self, n_clients: int, device=None, dtype=torch.float32) -> torch.Tensor:
        return torch.zeros(n_clients, self.size, dtype=dtype, device=device)

    def nbytes(self, dtype=torch.float32) -> int:
        return self.size * torch.tensor([], dtype=dtype).element_size()


def stack_state_dicts(layout: ParamLayout, state_dicts: List[Dict[str, torch.Tensor]], device=None) -> torch.Tensor:
    dev = device if device is not None else next(iter(state_dicts[0].values())).device
    out = layout.alloc_stack(len(state_dicts), dev)
    for i, sd in enumerate(state_dicts):
        layout.flatten(sd, out=out[i])
    return out


def fedavg_state_dicts(w_locals, device=None):
    """[(n_samples, state_dict)] → averaged state_dict through the flat arena + the FedAvg kernel.
    Unlike the reference `_aggregate` (Appendix A #10) the inputs are not mutated."""
    from ..ops import weighted_sum
    counts = [float(n) for n, _ in w_locals]
    total = sum(counts)
    sds = [sd for _, sd in w_locals]
    layout = ParamLayout(sds[0])
    dev = device if device is not None else next(iter(sds[0].values())).device
    stack = stack_state_dicts(layout, sds, dev)
    w = torch.tensor([c / total for c in counts], dtype=torch.float32, device=dev)
    avg = weighted_sum(stack, w)
    return layout.unflatten(avg)
