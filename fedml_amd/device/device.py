"""``get_device(args)`` (reference: `device/device.py:8-59`).

* single process / RCCL simulator: ``cuda:<gpu_id or LOCAL_RANK>`` if ``using_gpu`` and a GPU exists
* message-passing (MPI-style) simulation: ``gpu_mapping.yaml`` table
* hierarchical cross-silo: ``proc_rank_in_silo`` (torchrun LOCAL_RANK) → GPU
"""
import logging
import os

import torch

from .gpu_mapping import mapping_processes_to_gpu_device_from_yaml_file


def _gpu_ok(args):
    return bool(getattr(args, "using_gpu", False)) and torch.cuda.is_available()


def get_device(args):
    tt = getattr(args, "training_type", "simulation")
    backend = getattr(args, "backend", "single_process")
    if tt == "simulation" and backend in ("MPI", "TCP", "LOOPBACK") and getattr(args, "gpu_mapping_file", None):
        return mapping_processes_to_gpu_device_from_yaml_file(
            int(getattr(args, "process_id", 0)), int(getattr(args, "worker_num", 1)),
            args.gpu_mapping_file if _gpu_ok(args) else None, getattr(args, "gpu_mapping_key", None))
    if not _gpu_ok(args):
        return torch.device("cpu")
    n = torch.cuda.device_count()
    if tt == "cross_silo" and getattr(args, "scenario", "horizontal") == "hierarchical":
        idx = int(getattr(args, "rank_in_node", os.environ.get("LOCAL_RANK", 0)))
    elif "LOCAL_RANK" in os.environ:
        idx = int(os.environ["LOCAL_RANK"])
    else:
        idx = int(getattr(args, "gpu_id", 0))
    idx %= max(1, n)
    torch.cuda.set_device(idx)
    dev = torch.device(f"cuda:{idx}")
    logging.info("device = %s", dev)
    return dev
