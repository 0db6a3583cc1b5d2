"""Pickle-free wire format for Messages.

    frame := magic(4) | header_len(u32) | header JSON (utf-8, space-padded) | blob_0 | blob_1 | ...

The header is the message dict where every tensor / ndarray is replaced by
``{"__t__": i, "dtype": ..., "shape": [...], "off": byte_offset, "nbytes": n}`` pointing
into the blob area; dicts/lists nest. Nothing executable is ever deserialised (the reference pickles a
dict of tensors: `mpi_send_thread.py:27`, `grpc_comm_manager.py:68`).

Copies: ``encode_segments`` returns the frame as a list of buffers — the header plus a zero-copy view of
every CPU tensor (a device tensor costs its one device→host copy) — which the TCP transport writes
with one ``sendall`` per segment (no concatenation); ``decode`` of a writable buffer (the transport's
receive ``bytearray``) returns tensors that VIEW the frame (no per-tensor copy). Blobs start on 16-byte
boundaries of the frame, so every view is aligned.
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


_ALIGN = 16


def _add_blob(blobs, offset, raw) -> int:
    """Append ``raw`` (bytes-like) at the next 16-byte boundary of the blob area; returns its offset."""
    pad = -offset[0] % _ALIGN
    if pad:
        blobs.append(bytes(pad))
        offset[0] += pad
    at = offset[0]
    blobs.append(raw)
    offset[0] += len(raw)
    return at


def encode_obj(obj, blobs, offset):
    if isinstance(obj, torch.Tensor):
        t = obj.detach()
        if t.device.type != "cpu":
            t = t.cpu()
        t = t.contiguous()
        a = t.view(torch.int16).numpy() if t.dtype == torch.bfloat16 else t.numpy()
        raw = memoryview(a.reshape(-1)).cast("B")      # a view: the tensor's own bytes
        off = _add_blob(blobs, offset, raw)
        return {"__t__": "torch", "dtype": _dtype_name(t), "shape": list(t.shape), "off": off, "nbytes": len(raw)}
    if isinstance(obj, np.ndarray):
        a = np.ascontiguousarray(obj)
        if a.dtype == object:
            raise TypeError("object arrays are not serialisable (no pickle)")
        raw = memoryview(a.reshape(-1)).cast("B")
        off = _add_blob(blobs, offset, raw)
        return {"__t__": "numpy", "dtype": a.dtype.str, "shape": list(a.shape), "off": off, "nbytes": len(raw)}
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
        off = _add_blob(blobs, offset, obj)
        return {"__t__": "bytes", "off": off, "nbytes": len(obj)}
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
            writable = not raw.readonly   # views of a writable frame; a read-only frame is copied
            if kind == "numpy":
                arr = np.frombuffer(raw, dtype=np.dtype(obj["dtype"])).reshape(obj["shape"])
                return arr if writable else arr.copy()
            dt = _TORCH_DTYPES[obj["dtype"]]
            if obj["nbytes"] == 0:
                return torch.empty(obj["shape"], dtype=dt)
            if dt == torch.bfloat16:
                t = torch.frombuffer(raw if writable else bytearray(raw), dtype=torch.int16).view(torch.bfloat16)
            else:
                t = torch.frombuffer(raw if writable else bytearray(raw), dtype=dt)
            return t.reshape(obj["shape"])
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


def encode_segments(obj):
    """The frame as [head, blob views...] (see the module docstring) and its total length."""
    blobs = []
    header = json.dumps(encode_obj(obj, blobs, [0])).encode("utf-8")
    header += b" " * (-(8 + len(header)) % _ALIGN)     # the blob area starts on a 16-byte boundary
    segs = [MAGIC + struct.pack("<I", len(header)) + header] + blobs
    return segs, sum(len(b) for b in segs)


def encode(obj) -> bytes:
    segs, _ = encode_segments(obj)
    return b"".join(segs)


def decode(buf) -> object:
    mv = memoryview(buf)
    if bytes(mv[:4]) != MAGIC:
        raise ValueError("bad frame magic")
    (hl,) = struct.unpack("<I", mv[4:8])
    header = json.loads(bytes(mv[8:8 + hl]).decode("utf-8"))
    return decode_obj(header, mv[8 + hl:])


def encode_message(msg) -> bytes:
    return encode(msg.get_params())


def encode_message_segments(msg):
    return encode_segments(msg.get_params())


def decode_message(buf):
    from .message import Message
    m = Message()
    m.init(decode(buf))
    return m
