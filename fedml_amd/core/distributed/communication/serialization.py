"""Pickle-free wire format for Messages.

    frame := magic(4) | header_len(u32) | header JSON (utf-8) | blob_0 | blob_1 | ...

The header is the message dict where every tensor / ndarray is replaced by
``{"__t__": i, "dtype": ..., "shape": [...], "off": byte_offset, "nbytes": n}`` pointing
into the blob area; dicts/lists nest. state_dicts therefore cost one memcpy per tensor
(or one for a flat arena buffer), instead of the reference's pickle of a dict of tensors
(`mpi_send_thread.py:27`, `grpc_comm_manager.py:68`) — and nothing executable is ever
deserialised.
"""
import json
import struct
from collections import OrderedDict

import numpy as np
import torch

MAGIC = b"FAM1"

_TORCH_DTYPES = {
    "float32": torch.float32, "float64": torch.float64, "float16": torch.float16, "bfloat16": torch.bfloat16,
    "int64": torch.int64, "int32": torch.int32, "int16": torch.int16, "int8": torch.int8, "uint8": torch.uint8,
    "bool": torch.bool,
}


def _dtype_name(t: torch.Tensor) -> str:
    return str(t.dtype).replace("torch.", "")


def encode_obj(obj, blobs, offset):
    if isinstance(obj, torch.Tensor):
        t = obj.detach()
        if t.device.type != "cpu":
            t = t.cpu()
        t = t.contiguous()
        if t.dtype == torch.bfloat16:
            raw = t.view(torch.int16).numpy().tobytes()
        else:
            raw = t.numpy().tobytes()
        desc = {"__t__": "torch", "dtype": _dtype_name(t), "shape": list(t.shape), "off": offset[0],
                "nbytes": len(raw)}
        blobs.append(raw)
        offset[0] += len(raw)
        return desc
    if isinstance(obj, np.ndarray):
        a = np.ascontiguousarray(obj)
        if a.dtype == object:
            raise TypeError("object arrays are not serialisable (no pickle)")
        raw = a.tobytes()
        desc = {"__t__": "numpy", "dtype": a.dtype.str, "shape": list(a.shape), "off": offset[0], "nbytes": len(raw)}
        blobs.append(raw)
        offset[0] += len(raw)
        return desc
    if isinstance(obj, dict):
        kind = "od" if isinstance(obj, OrderedDict) else "d"
        return {"__d__": kind, "items": [[encode_obj(k, blobs, offset), encode_obj(v, blobs, offset)]
                                         for k, v in obj.items()]}
    if isinstance(obj, (list, tuple)):
        return {"__l__": "t" if isinstance(obj, tuple) else "l", "items": [encode_obj(v, blobs, offset) for v in obj]}
    if isinstance(obj, (np.integer,)):
        return int(obj)
    if isinstance(obj, (np.floating,)):
        return float(obj)
    if isinstance(obj, bytes):
        desc = {"__t__": "bytes", "off": offset[0], "nbytes": len(obj)}
        blobs.append(obj)
        offset[0] += len(obj)
        return desc
    if obj is None or isinstance(obj, (int, float, str, bool)):
        return obj
    raise TypeError(f"cannot serialise {type(obj).__name__} (no pickle on the wire)")


def decode_obj(obj, blob: memoryview):
    if isinstance(obj, dict):
        if "__t__" in obj:
            kind = obj["__t__"]
            raw = blob[obj["off"]:obj["off"] + obj["nbytes"]]
            if kind == "bytes":
                return bytes(raw)
            if kind == "numpy":
                return np.frombuffer(raw, dtype=np.dtype(obj["dtype"])).reshape(obj["shape"]).copy()
            dt = _TORCH_DTYPES[obj["dtype"]]
            if dt == torch.bfloat16:
                arr = np.frombuffer(raw, dtype=np.int16).copy()
                return torch.from_numpy(arr).view(torch.bfloat16).reshape(obj["shape"])
            npdt = torch.empty(0, dtype=dt).numpy().dtype
            arr = np.frombuffer(raw, dtype=npdt).copy()
            return torch.from_numpy(arr).reshape(obj["shape"])
        if "__d__" in obj:
            d = OrderedDict() if obj["__d__"] == "od" else {}
            for k, v in obj["items"]:
                d[decode_obj(k, blob)] = decode_obj(v, blob)
            return d
        if "__l__" in obj:
            items = [decode_obj(v, blob) for v in obj["items"]]
            return tuple(items) if obj["__l__"] == "t" else items
        return {k: decode_obj(v, blob) for k, v in obj.items()}
    return obj


def encode(obj) -> bytes:
    blobs = []
    header = json.dumps(encode_obj(obj, blobs, [0])).encode("utf-8")
    return MAGIC + struct.pack("<I", len(header)) + header + b"".join(blobs)


def decode(buf) -> object:
    mv = memoryview(buf)
    if bytes(mv[:4]) != MAGIC:
        raise ValueError("bad frame magic")
    (hl,) = struct.unpack("<I", mv[4:8])
    header = json.loads(bytes(mv[8:8 + hl]).decode("utf-8"))
    return decode_obj(header, mv[8 + hl:])


def encode_message(msg) -> bytes:
    return encode(msg.get_params())


def decode_message(buf):
    from .message import Message
    m = Message()
    m.init(decode(buf))
    return m
