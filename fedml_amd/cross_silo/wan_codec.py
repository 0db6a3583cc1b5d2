"""Compressed model uploads on the cross-silo WAN path.

The reference ships every silo's full fp32 state_dict to the server each round
(``cross_silo/horizontal/utils.py:7-18``, ``client_manager.py`` send_model_to_server). With
``wan_compression: int8`` a silo instead uploads its UPDATE Δ = w_local − w_global as ONE flat
block-256 int8 buffer with per-block fp32 scales (the ``fa_quant_int8`` HIP kernel: stochastic
rounding + per-silo error feedback — the quantisation error is carried into the next round's
update, so it is not lost), ≈ 3.9× fewer bytes than fp32. Non-float entries
(``num_batches_tracked``) travel raw. The server reconstructs w_global + deq(Δ) before FedAvg,
so the aggregator, robust-aggregation hooks and FedOpt are unchanged.

Wire format (pickle-free ``serialization``): ``{"__wan_codec__": "int8", "q": int8[n],
"s": f32[ceil(n/256)], "n": n, "raw": {key: tensor}}``; float keys in state_dict order."""
from collections import OrderedDict
from typing import Dict, Optional

import torch

from ..ops.fl_ops import dequantize_int8_axpy, quantize_int8

CODEC_KEY = "__wan_codec__"


def _float_keys(sd):
    return [k for k, v in sd.items() if torch.is_tensor(v) and v.is_floating_point()]


def flatten_float(sd, device=None) -> torch.Tensor:
    ks = _float_keys(sd)
    if not ks:
        return torch.zeros(0)
    return torch.cat([sd[k].detach().reshape(-1).to(device=device, dtype=torch.float32) for k in ks])


def payload_bytes(obj) -> int:
    """Tensor bytes of a (nested) message payload — what the WAN carries besides the header."""
    if torch.is_tensor(obj):
        return obj.numel() * obj.element_size()
    if isinstance(obj, dict):
        return sum(payload_bytes(v) for v in obj.values())
    if isinstance(obj, (list, tuple)):
        return sum(payload_bytes(v) for v in obj)
    return 0


def is_encoded(obj) -> bool:
    return isinstance(obj, dict) and CODEC_KEY in obj


class WanEncoder:
    """Silo side: remembers the global model of the round and the error-feedback residual."""

    def __init__(self, method: str = "int8", device=None):
        if method != "int8":
            raise ValueError(f"wan_compression {method!r}: expected int8")
        self.method = method
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.ref: Optional[torch.Tensor] = None
        self.residual: Optional[torch.Tensor] = None
        self.calls = 0

    def note_global(self, sd):
        if sd is not None:
            self.ref = flatten_float(sd, self.device)

    def encode(self, sd, seed: int = 0) -> Dict:
        flat = flatten_float(sd, self.device)
        if self.ref is None or self.ref.numel() != flat.numel():
            raise RuntimeError("WanEncoder.encode before the round's global model was noted")
        if self.residual is None:
            self.residual = torch.zeros_like(flat)
        self.calls += 1
        q, s = quantize_int8(flat - self.ref, residual=self.residual, stochastic=True,
                             seed=(int(seed) * 1000003 + self.calls) & 0x7FFFFFFF)
        raw = OrderedDict((k, v) for k, v in sd.items() if not (torch.is_tensor(v) and v.is_floating_point()))
        return {CODEC_KEY: self.method, "q": q.cpu(), "s": s.cpu(), "n": int(flat.numel()), "raw": raw}


def decode(payload: Dict, global_sd, device=None) -> "OrderedDict[str, torch.Tensor]":
    """Server side: w_global + deq(Δ) as a state_dict shaped like ``global_sd``."""
    if payload.get(CODEC_KEY) != "int8":
        raise ValueError(f"unknown WAN codec {payload.get(CODEC_KEY)!r}")
    dev = torch.device(device) if device is not None else torch.device("cpu")
    acc = flatten_float(global_sd, dev).clone()
    if acc.numel() != int(payload["n"]):
        raise ValueError("WAN payload does not match the global model")
    dequantize_int8_axpy(payload["q"].to(dev), payload["s"].to(dev), 1.0, acc)
    out, off = OrderedDict(), 0
    for k, v in global_sd.items():
        if torch.is_tensor(v) and v.is_floating_point():
            n = v.numel()
            out[k] = acc[off:off + n].view_as(v).to(v.dtype).to(v.device)
            off += n
        else:
            out[k] = payload["raw"].get(k, v)
    return out
