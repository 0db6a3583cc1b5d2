"""Collectives over RCCL (xGMI) — one process per GPU, ``torch.distributed`` backend ``nccl``
(= RCCL on ROCm); ``gloo`` on CPU for tests.

Design for xGMI (7 point-to-point links per MI355X, ~153 GB/s each): FL payloads are
small (ResNet-56 = 2.46 MB), so a round is latency-bound → ONE flat buffer per GPU per
round (model + sample count packed together), never per-tensor/per-client messages.
Large payloads (DistilBERT / ViT, 130-350 MB) are split into a few big buckets issued
on a dedicated communication stream so they overlap the tail of local training.
"""
import datetime
import logging
import os
from typing import List, Optional

import torch
import torch.distributed as dist

_COMM_STREAMS = {}


def init_process_group(backend: Optional[str] = None, timeout_s: int = 1800, device=None, args=None):
    """Idempotent init from torchrun env (RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT).

    ``args`` (the run config) is read before the group exists: ``deterministic`` pins the RCCL algorithm and
    protocol; ``elastic`` makes a dead peer surface as an exception in the survivors instead of a hang —
    the group gets the ``elastic_timeout_s`` timeout, and under RCCL every collective wait blocks with that
    timeout (``TORCH_NCCL_BLOCKING_WAIT``) while the watchdog aborts the broken communicator without
    tearing the process down (``TORCH_NCCL_ASYNC_ERROR_HANDLING=2``, clean-up only) — the simulator then
    rebuilds the group from the survivors (``parallel.elastic``)."""
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world <= 1:
        return 0, 1
    if backend is None:
        # FEDML_AMD_DIST_BACKEND=gloo rehearses multi-rank GPU runs on a box with fewer GPUs than
        # ranks (RCCL needs one GPU per rank); production runs use RCCL ("nccl" on ROCm)
        backend = os.environ.get("FEDML_AMD_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    from ..utils import determinism
    determinism.apply_env(args)     # deterministic mode: fixed RCCL algorithm / protocol
    if args is not None and bool(getattr(args, "elastic", False)):
        timeout_s = int(getattr(args, "elastic_timeout_s", 60) or 60)
        if backend == "nccl":
            os.environ["TORCH_NCCL_BLOCKING_WAIT"] = "1"
            os.environ["TORCH_NCCL_ASYNC_ERROR_HANDLING"] = "2"
    kw = {}
    if backend == "nccl" and device is not None:
        kw["device_id"] = torch.device(device)
    dist.init_process_group(backend=backend, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)
    logging.info("process group up: rank %d/%d backend=%s", rank, world, backend)
    return rank, world


def backend_name() -> str:
    """Human label of the active collective backend: RCCL (``nccl`` on ROCm), gloo, or none."""
    if not (dist.is_available() and dist.is_initialized()):
        return "none"
    b = str(dist.get_backend())
    return "RCCL" if b == "nccl" else b


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def rank() -> int:
    return dist.get_rank() if is_dist() else 0


def world_size() -> int:
    return dist.get_world_size() if is_dist() else 1


def comm_stream(device) -> Optional[torch.cuda.Stream]:
    if torch.device(device).type != "cuda":
        return None
    key = str(device)
    if key not in _COMM_STREAMS:
        _COMM_STREAMS[key] = torch.cuda.Stream(device=device, priority=-1)
    return _COMM_STREAMS[key]


def _host_staged(buf: torch.Tensor, group=None) -> bool:
    """gloo on device tensors (multi-rank rehearsals on a box with fewer GPUs than ranks): the collective runs on
    a host copy — ``.cpu()`` orders it after every kernel that produced the buffer and the copy back is ordered
    before every later kernel on this stream, with no reliance on gloo's internal device-stream handoff."""
    return buf.is_cuda and str(dist.get_backend(group)) == "gloo"


def all_reduce_flat(buf: torch.Tensor, group=None, bucket_bytes: int = 64 << 20, async_op: bool = False):
    """SUM all-reduce of a flat buffer in ≤ ``bucket_bytes`` slices (one slice for FL-sized models)."""
    if not is_dist():
        return [] if async_op else buf
    if _host_staged(buf, group):
        h = buf.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
        buf.copy_(h)
        return [] if async_op else buf
    n = buf.numel()
    per = max(1, bucket_bytes // buf.element_size())
    works = []
    for s in range(0, n, per):
        works.append(dist.all_reduce(buf[s:s + per], op=dist.ReduceOp.SUM, group=group, async_op=True))
    if async_op:
        return works
    for w in works:
        w.wait()
    return buf


def broadcast_flat(buf: torch.Tensor, src: int = 0, group=None):
    if is_dist():
        if _host_staged(buf, group):
            h = buf.cpu()
            dist.broadcast(h, src=src, group=group)
            buf.copy_(h)
        else:
            dist.broadcast(buf, src=src, group=group)
    return buf


def reduce_flat(buf: torch.Tensor, dst: int = 0, group=None):
    if is_dist():
        if _host_staged(buf, group):
            h = buf.cpu()
            dist.reduce(h, dst=dst, op=dist.ReduceOp.SUM, group=group)
            buf.copy_(h)
        else:
            dist.reduce(buf, dst=dst, op=dist.ReduceOp.SUM, group=group)
    return buf


def all_gather_flat(buf: torch.Tensor, group=None) -> List[torch.Tensor]:
    if not is_dist():
        return [buf]
    if _host_staged(buf, group):
        h = buf.cpu()
        out = [torch.empty_like(h) for _ in range(world_size())]
        dist.all_gather(out, h, group=group)
        return [o.to(buf.device) for o in out]
    out = [torch.empty_like(buf) for _ in range(world_size())]
    dist.all_gather(out, buf, group=group)
    return out


def barrier(device=None):
    if is_dist():
        if device is not None and torch.device(device).type == "cuda" and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.device(device).index])
        else:
            dist.barrier()


def max_over_ranks(value: float, device) -> float:
    if not is_dist():
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64 if torch.device(device).type == "cpu" else torch.float32,
                     device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def destroy():
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
