"""Intra-silo process group (reference: `cross_silo/hierarchical/process_group_manager.py:8-45`):
the silo's processes rendezvous on their own TCP store (``pg_master_address:pg_master_port``) so
the group is independent of any other torch.distributed world; backend RCCL (``nccl``) on GPUs,
gloo on CPU."""
import datetime
import logging
import os

import torch
import torch.distributed as dist


class ProcessGroupManager:
    def __init__(self, rank, world_size, master_address="127.0.0.1", master_port=29700, only_gpu=None,
                 timeout_s=1800):
        self.rank, self.world_size = int(rank), int(world_size)
        use_gpu = torch.cuda.is_available() if only_gpu is None else bool(only_gpu)
        # FEDML_AMD_DIST_BACKEND=gloo: rehearsal with several silo processes sharing one GPU
        backend = os.environ.get("FEDML_AMD_DIST_BACKEND") or ("nccl" if use_gpu else "gloo")
        if not dist.is_initialized():
            dist.init_process_group(backend=backend, init_method=f"tcp://{master_address}:{int(master_port)}",
                                    rank=self.rank, world_size=self.world_size,
                                    timeout=datetime.timedelta(seconds=timeout_s))
        logging.info("silo process group: rank %d/%d (%s)", self.rank, self.world_size, backend)
        self.messenger_group = None

    def get_process_group(self):
        return dist.group.WORLD

    def cleanup(self):
        if dist.is_initialized():
            dist.destroy_process_group()
