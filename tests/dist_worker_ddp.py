"""Worker for tests/test_ddp.py: FlatDDP on CPU/gloo vs. a single-process full-batch reference
(FEDML_TEST_DEVICE=cuda: both ranks on cuda:0 — FlatDDP's comm stream, HIP optimizer kernels and
bucket hooks on the GPU, collectives over gloo because the box has one GPU)."""
import os
import sys

import torch
import torch.nn as nn


def main(rank, world, port, out, mode="flat"):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fedml_amd.distributed import FlatDDP, FlatOptimizer
    dev = os.environ.get("FEDML_TEST_DEVICE", "cpu")
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(12, 32), nn.ReLU(), nn.Linear(32, 32), nn.ReLU(), nn.Linear(32, 5)).to(dev)
    ddp = FlatDDP(model, dev, bucket_mb=0.002)  # tiny buckets → several overlapping all-reduces
    opt = FlatOptimizer(ddp, "sgd", lr=0.1, momentum=0.9) if mode == "flat" else \
        torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9)
    g = torch.Generator().manual_seed(1)
    X = torch.randn(4 * 8, 12, generator=g)
    Y = torch.randint(0, 5, (4 * 8,), generator=g)
    for step in range(3):
        xs, ys = X.view(4, 8, 12)[step % 4], Y.view(4, 8)[step % 4]
        per = 8 // world
        x, y = xs[rank * per:(rank + 1) * per].to(dev), ys[rank * per:(rank + 1) * per].to(dev)
        opt.zero_grad()  # torch optimizers set grads to None: FlatDDP re-homes them
        nn.functional.cross_entropy(ddp(x), y).backward()  # all-reduce completes at end of backward
        opt.step()
    if rank == 0:
        torch.save({k: v.detach().cpu().clone() for k, v in model.state_dict().items()}, out)
    dist.destroy_process_group()


if __name__ == "__main__":
    import mp_harness
    mp_harness.install_stack_dump()
    main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5])
