"""Worker for the sharded decentralized-gossip test: rank world port out mode."""
import os
import sys

import torch


def main(rank, world, port, out, mode):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from fedml_amd.arguments import Arguments
    from fedml_amd.models.linear.lr import LogisticRegression
    from fedml_amd.parallel import comm
    from fedml_amd.simulation.sp.decentralized.decentralized_api import DecentralizedFLAPI
    if world > 1:
        comm.init_process_group(backend="gloo")
    g = torch.Generator().manual_seed(0)
    N, T, d = 6, 20, 10
    X = torch.randn(N, T, d, generator=g)
    Y = (X[..., 0] > 0).long()
    args = Arguments.from_dict({"x": {"client_num_in_total": N, "iteration_number": T, "mode": mode,
                                      "learning_rate": 0.1, "b_symmetric": mode != "PUSHSUM",
                                      "topology_neighbors_num_undirected": 2, "topology_neighbors_num_directed": 2,
                                      "epoch": 1}})
    torch.manual_seed(1)
    import numpy as np
    np.random.seed(0)   # the asymmetric topology draws random edges
    api = DecentralizedFLAPI(args, torch.device("cpu"), (X, Y), LogisticRegression(d, 2))
    res = api.train()
    if rank == 0:
        torch.save({"params": res["params"], "regret": torch.tensor(res["regret"])}, out)
    comm.destroy()


if __name__ == "__main__":
    import mp_harness
    mp_harness.install_stack_dump()
    main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], sys.argv[5])
