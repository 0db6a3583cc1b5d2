"""Error/lock helpers (reference: `utils/context.py:8-38`).

The reference's ``raise_MPI_error`` aborts ``MPI.COMM_WORLD`` on any exception.
Here the equivalent aborts the torch.distributed process group (RCCL/gloo)
so peers do not hang, then re-raises.
"""
import contextlib
import logging
import os
import threading
import traceback

_locks = {}


@contextlib.contextmanager
def raise_error_and_retry(abort_group: bool = True):
    try:
        yield
    except Exception:
        logging.error(traceback.format_exc())
        if abort_group:
            try:
                import torch.distributed as dist
                if dist.is_available() and dist.is_initialized():
                    dist.destroy_process_group()
            except Exception:
                pass
        raise


# alias used by reference code
raise_MPI_error = raise_error_and_retry


def get_lock(name: str = "default") -> threading.Lock:
    lk = _locks.get(name)
    if lk is None:
        lk = _locks.setdefault(name, threading.Lock())
    return lk


def post_complete_message_to_sweep_process(args, path="./tmp/fedml"):
    """Write a completion line into the sweep FIFO/file (reference: `cross_silo/horizontal/utils.py:21-29`)."""
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "a") as f:
        f.write("training is finished! \n%s\n" % (str(getattr(args, "run_id", "0"))))
