"""Communicator abort / re-init for the RCCL simulator (fault tolerance and elasticity).

The reference has no collective failure handling (an MPI rank that dies hangs the job). Here a
collective that fails — a peer process died: the gloo/RCCL transport raises instead of completing — is
caught by the simulator, the broken process group is torn down and the SURVIVORS rendezvous again on a
side TCP store (hosted by rank 0, which must survive; it is the coordinator, like the reference's
server): every survivor checks in under a new generation key, waits ``settle_s`` for late arrivals, and
re-initialises the process group with the ranks that checked in, in arrival order. The simulator then
re-packs the round's clients over the new world (``pack_clients_to_gpus``) and repeats the round from the
unchanged global model — results are world-size invariant, so the run continues as if it had started
with the smaller world."""
import datetime
import logging
import os
import time

import torch
import torch.distributed as dist

_STATE = {"store": None, "gen": 0, "backend": None, "timeout": 60}


def enabled() -> bool:
    return _STATE["store"] is not None


def setup(rank: int, world: int, backend: str, timeout_s: int = 60, port: int = None):
    """Open the side store (rank 0 hosts it) before any failure can happen."""
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(port or int(os.environ.get("MASTER_PORT", "29500")) + 1)
    _STATE["store"] = dist.TCPStore(addr, port, world, is_master=(rank == 0),
                                    timeout=datetime.timedelta(seconds=max(timeout_s, 30)), wait_for_workers=False)
    _STATE["backend"], _STATE["timeout"] = backend, timeout_s


def reinit(settle_s: float = 3.0):
    """Tear down the broken group and rebuild it from the survivors. Returns (new_rank, new_world)."""
    st = _STATE["store"]
    if st is None:
        raise RuntimeError("elastic.setup() was not called")
    try:
        if dist.is_initialized():
            dist.destroy_process_group()
    except Exception as e:   # a broken communicator may not tear down cleanly
        logging.warning("elastic: destroy_process_group failed (%s)", e)
    _STATE["gen"] += 1
    g = _STATE["gen"]
    idx = int(st.add(f"elastic/{g}/arrived", 1)) - 1
    if idx == 0:
        # the first survivor closes the generation once nobody new has checked in for settle_s (peers detect
        # the failure at different times — a loaded machine spreads that by seconds)
        last, quiet = 1, 0.0
        while quiet < settle_s:
            time.sleep(0.2)
            n = int(st.add(f"elastic/{g}/arrived", 0))
            quiet = 0.0 if n != last else quiet + 0.2
            last = n
        st.set(f"elastic/{g}/world", str(last))
    world = int(st.get(f"elastic/{g}/world"))   # blocks until the generation is closed
    if idx >= world:
        raise RuntimeError("elastic: arrived after the new world was fixed")
    pg_store = dist.PrefixStore(f"elastic/{g}/pg", st)
    dist.init_process_group(_STATE["backend"], store=pg_store, rank=idx, world_size=world,
                            timeout=datetime.timedelta(seconds=_STATE["timeout"]))
    logging.warning("elastic: generation %d — rank %d of %d survivors", g, idx, world)
    return idx, world
