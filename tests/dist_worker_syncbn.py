"""Worker for the SyncBN test: rank world port out — each rank normalises its half of the batch."""
import os
import sys

import torch


def main(rank, world, port, out):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from fedml_amd.models.cv.batchnorm_utils import convert_sync_batchnorm
    from fedml_amd.parallel import comm
    comm.init_process_group(backend="gloo")
    g = torch.Generator().manual_seed(0)
    x = torch.randn(8, 6, 5, 5, generator=g) * 3 + 1
    dy = torch.randn(8, 6, 5, 5, generator=g)
    bn = torch.nn.BatchNorm2d(6)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5, generator=g)
        bn.bias.uniform_(-0.5, 0.5, generator=g)
    sbn = convert_sync_batchnorm(torch.nn.Sequential(bn))
    per = 8 // world
    xs = x[rank * per:(rank + 1) * per].clone().requires_grad_(True)
    y = sbn(xs)
    y.backward(dy[rank * per:(rank + 1) * per])
    w_g = sbn[0].weight.grad.clone()
    b_g = sbn[0].bias.grad.clone()
    comm.all_reduce_flat(w_g)
    comm.all_reduce_flat(b_g)
    parts = comm.all_gather_flat(torch.cat([y.detach().reshape(-1), xs.grad.reshape(-1)]))
    if rank == 0:
        torch.save({"parts": parts, "wg": w_g, "bg": b_g, "rm": sbn[0].running_mean, "rv": sbn[0].running_var}, out)
    comm.destroy()


if __name__ == "__main__":
    import mp_harness
    mp_harness.install_stack_dump()
    main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
