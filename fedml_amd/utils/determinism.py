"""Deterministic mode (SURVEY §5.2 "a deterministic mode (fixed reduction order)").

``enable()`` (``deterministic: true`` in the config, or ``FEDML_AMD_DETERMINISTIC=1``) makes a run bitwise
reproducible from run to run on the same world size:

* collectives: RCCL pinned to one algorithm and protocol (``NCCL_ALGO=Ring``, ``NCCL_PROTO=Simple``) —
  the ring visits ranks in a fixed order, so every all-reduce sums in the same order every run (set
  before the process group is created; ``parallel.comm.init_process_group`` calls ``apply_env()``);
* FL aggregation kernels are fixed-order by construction (``fl_kernels.hip``: the weighted sum walks the
  clients in slot order per element; norms use fixed partial slots + an ordered finalize);
* the client-batched ResNet step keeps the native HIP kernels: their cross-workgroup fp32 atomics (BN
  statistics, split weight gradients) accumulate into 128-bit fixed-point shadows instead and are rounded
  once (``ops/det_ops.py``, ``csrc/detacc.h``); the tiling of those kernels is fixed independently of the
  number of client slots per GPU, so a client's gradients do not depend on the world size either;
* the fp32 transformer kernels' LayerNorm / bias-gradient reductions become fixed-order column sums;
* the aggregation partial sums Σ n_c·w_c (and their all-reduce) run in fp64 and are rounded to fp32
  once, so packing clients onto more ranks does not change the global model's bits;
* data order / augmentation / dropout are already keyed by (seed, round, client id).

The cost is the native conv speed-up; deterministic runs are for debugging and bisecting, not benchmarks.
"""
import os

import torch

_ENABLED = [os.environ.get("FEDML_AMD_DETERMINISTIC", "0") == "1"]


def enabled(args=None) -> bool:
    if args is not None and bool(getattr(args, "deterministic", False)):
        return True
    return _ENABLED[0]


def apply_env(args=None):
    """Collective-library settings that fix the reduction order (call before the process group exists)."""
    if enabled(args):
        os.environ["NCCL_ALGO"] = "Ring"
        os.environ["NCCL_PROTO"] = "Simple"


def enable(args=None):
    _ENABLED[0] = True
    if args is not None:
        args.deterministic = True
    apply_env()
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
    # cuBLAS/hipBLASLt workspace config required for deterministic GEMMs
    os.environ.setdefault("CUBLAS_WORKSPACE_CONFIG", ":4096:8")


def disable():
    """Leave deterministic mode (tests; a process normally keeps one mode for its lifetime)."""
    _ENABLED[0] = False
    torch.use_deterministic_algorithms(False)
    torch.backends.cudnn.deterministic = False
    for k in ("NCCL_ALGO", "NCCL_PROTO"):
        os.environ.pop(k, None)
