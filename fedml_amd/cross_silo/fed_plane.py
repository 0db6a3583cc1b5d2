"""RCCL data plane between the cross-silo server and the silo masters on one node (``silo_transport: rccl``).

The reference ships every model between the server and the silo masters as a pickled / JSON state dict over the
network transport (`cross_silo/hierarchical/client_master_manager.py:239-249`, `horizontal/fedml_server_manager.py:
121-207`). On one MI355X node the server and the silo masters instead share ONE standalone communicator — rank 0 the
server, rank k the master of the k-th silo of ``client_id_list`` — built directly on a TCP store
(``ProcessGroupNCCL`` = RCCL over xGMI; gloo for rehearsals with several ranks on one GPU) and independent of each
silo's own process group (`process_group_manager.py`, the intra-silo data parallelism keeps its default group):

    round r   server: markers to EVERY silo (TCP) → broadcast(global [P])      ─┐ one flat collective each way
              master: broadcast → (selected: train → C2S marker) → reduce(n·w ‖ n) ─┘ (unselected silos add zeros)
              server: after every selected silo's marker → reduce → w = Σ n·w / Σ n

Every master joins every round's two collectives (partial participation included), so the collective sequence is
the same on every rank; the control transport keeps the handshake, the round index and the data-silo assignment.
Deadline rounds are not supported on this plane (a missing silo would stall the collective)."""
import datetime
import logging
import os

import torch
import torch.distributed as dist
from torch._C._distributed_c10d import BroadcastOptions, ReduceOp, ReduceOptions, AllreduceOptions


class FederationPlane:
    def __init__(self, rank: int, size: int, port: int, device, host: str = "127.0.0.1", timeout_s: int = 1800):
        self.rank, self.size = int(rank), int(size)
        self.device = torch.device(device)
        timeout = datetime.timedelta(seconds=timeout_s)
        self._tcp = dist.TCPStore(host, int(port), self.size, self.rank == 0, timeout)
        store = dist.PrefixStore("fedml_amd_fed_plane", self._tcp)
        # RCCL needs one GPU per rank: with more plane ranks than GPUs (a one-GPU rehearsal, 8 silos + the server on
        # an 8-GPU node) the launcher picks gloo (FEDML_AMD_PLANE_BACKEND / FEDML_AMD_DIST_BACKEND)
        backend = (os.environ.get("FEDML_AMD_PLANE_BACKEND") or os.environ.get("FEDML_AMD_DIST_BACKEND")
                   or ("nccl" if self.device.type == "cuda" else "gloo"))
        self.backend = backend
        if backend == "nccl":
            from torch._C._distributed_c10d import ProcessGroupNCCL
            torch.cuda.set_device(self.device)
            self.pg = ProcessGroupNCCL(store, self.rank, self.size, timeout)
        else:
            from torch._C._distributed_c10d import ProcessGroupGloo
            self.pg = ProcessGroupGloo(store, self.rank, self.size, timeout)
        logging.info("federation plane up: rank %d/%d (%s)", self.rank, self.size, backend)

    def broadcast(self, t: torch.Tensor) -> torch.Tensor:
        """The server's ``t`` into every rank's ``t`` (in place)."""
        opts = BroadcastOptions()
        opts.rootRank = 0
        self.pg.broadcast([t], opts).wait()
        return t

    def reduce(self, t: torch.Tensor) -> torch.Tensor:
        """Σ over ranks of ``t`` into the server's ``t`` (RCCL reduce; gloo rehearsals all-reduce — its reduce takes
        host tensors only)."""
        if self.backend == "nccl":
            opts = ReduceOptions()
            opts.rootRank = 0
            opts.reduceOp = ReduceOp.SUM
            self.pg.reduce([t], opts).wait()
        else:
            opts = AllreduceOptions()
            opts.reduceOp = ReduceOp.SUM
            self.pg.allreduce([t], opts).wait()
        return t

    def close(self):
        """Shut the communicator down and release the store (its TCP port) — called from the managers' finish()."""
        pg, self.pg = self.pg, None
        if pg is not None and hasattr(pg, "shutdown"):
            try:
                pg.shutdown()
            except Exception as e:  # noqa: BLE001 - teardown is best effort
                logging.debug("federation plane shutdown: %s", e)
        self._tcp = None


def plane_port(args) -> int:
    """``fed_plane_port`` if configured, else a free port picked on the server (the markers carry it to the silo
    masters): concurrent cross-silo runs on one node, or a second run in the same process, never share a store."""
    p = int(getattr(args, "fed_plane_port", 0) or 0)
    if p:
        return p
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])
