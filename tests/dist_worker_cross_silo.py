"""Worker for the hierarchical cross-silo test: role ∈ {server, silo}."""
import copy
import logging
import sys

import torch


def main(role, silo, rank_in_silo, pg_port, out):
    import fedml_amd
    from fedml_amd.arguments import Arguments
    torch.set_num_threads(1)
    cfg = {"training_type": "cross_silo", "scenario": "hierarchical", "dataset": "mnist", "model": "lr",
           "client_num_in_total": 2, "client_num_per_round": 2, "comm_round": 2, "epochs": 1, "batch_size": 8,
           "learning_rate": 0.05, "frequency_of_the_test": 1, "backend": "TCP", "federated_optimizer": "FedAvg",
           "worker_num": 3, "client_id_list": "[1, 2]", "sys_perf_interval": 0, "synthetic_samples_per_client": 48,
           "rank": silo, "n_proc_in_silo": 2, "proc_rank_in_silo": rank_in_silo, "pg_master_port": pg_port}
    args = fedml_amd.init(Arguments.from_dict({"x": cfg}))
    logging.getLogger().setLevel(logging.WARNING)
    dev, ds, m = fedml_amd._prepare(args)
    from fedml_amd.cross_silo.hierarchical import Client, Server
    if role == "server":
        g = Server(args, dev, ds, m).run()
        torch.save(g, out)
    else:
        Client(args, dev, ds, m).run()


if __name__ == "__main__":
    import mp_harness
    mp_harness.install_stack_dump()
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5])
