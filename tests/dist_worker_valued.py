"""Worker for tests/test_valued_rccl.py::test_valued_rccl_two_ranks_equal_one_rank: one rank of the S-FedAvg RCCL
simulator on CPU/gloo. Rank 0 saves the sampled ids, φ per round and the final global flat model."""
import logging
import os
import sys

import numpy as np
import torch


def main(rank, world, port, out):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": str(port)})
    torch.set_num_threads(1)
    import fedml_amd
    from fedml_amd.arguments import Arguments
    from fedml_amd.parallel import comm
    from fedml_amd.simulation.rccl.valued import ValuedRCCLSimulator
    cfg = {"training_type": "simulation", "dataset": "mnist", "model": "lr", "client_num_in_total": 8,
           "client_num_per_round": 5, "comm_round": 3, "epochs": 1, "batch_size": 16, "learning_rate": 0.1,
           "frequency_of_the_test": 0, "backend": "RCCL", "federated_optimizer": "S-FedAvg",
           "synthetic_train_samples_per_client": 64, "partition_method": "hetero", "valid_samples": 200,
           "shuffle": True, "random_seed": 0}
    a = fedml_amd.init(Arguments.from_dict({"x": cfg}))
    logging.getLogger().setLevel(logging.WARNING)
    dev, ds, m = fedml_amd._prepare(a)
    np.random.seed(0)
    sim = ValuedRCCLSimulator(a, "cpu", ds, m)
    sim.run()
    if rank == 0:
        torch.save({"sampled": sim.results["sampled"], "phi": sim.results["phi"],
                    "w": sim.global_flat.detach().clone()}, out)
    sim.close()
    comm.destroy()


if __name__ == "__main__":
    import mp_harness
    mp_harness.install_stack_dump()
    main(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
