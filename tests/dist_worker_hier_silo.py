"""Worker for the batched-silo hierarchical cross-silo tests: role ∈ {server, silo}.
argv: role silo rank_in_silo pg_port out n_proc n_local device [model dataset rounds]"""
import logging
import os
import sys

import torch


def main(role, silo, rank_in_silo, pg_port, out, n_proc, n_local, device, model="lr", dataset="mnist", rounds=2,
         n_silos=2):
    import fedml_amd
    from fedml_amd.arguments import Arguments
    torch.set_num_threads(1)
    cfg = {"training_type": "cross_silo", "scenario": "hierarchical", "dataset": dataset, "model": model,
           "client_num_in_total": n_silos,
           "client_num_per_round": int(os.environ.get("FEDML_TEST_PER_ROUND", n_silos)), "comm_round": rounds, "epochs": 1,
           "batch_size": 8, "learning_rate": 0.05, "frequency_of_the_test": 0, "backend": "TCP",
           "federated_optimizer": "FedAvg", "worker_num": n_silos + 1,
           "client_id_list": str(list(range(1, n_silos + 1))), "sys_perf_interval": 0,
           "synthetic_samples_per_client": 48, "rank": silo, "n_proc_in_silo": n_proc,
           "proc_rank_in_silo": rank_in_silo, "pg_master_port": pg_port, "silo_local_clients": n_local,
           "shuffle": False, "using_gpu": device == "cuda", "gpu_id": 0,
           "silo_transport": os.environ.get("FEDML_TEST_SILO_TRANSPORT", ""),
           "fed_plane_port": int(os.environ.get("FEDML_TEST_PLANE_PORT", "0"))}
    args = fedml_amd.init(Arguments.from_dict({"x": cfg}))
    logging.getLogger().setLevel(logging.WARNING)
    dev, ds, m = fedml_amd._prepare(args)
    from fedml_amd.cross_silo.hierarchical import Client, Server
    if role == "server":
        g = Server(args, dev, ds, m).run()
        torch.save({k: v.cpu() for k, v in g.items()}, out)
    else:
        Client(args, dev, ds, m).run()


if __name__ == "__main__":
    import mp_harness
    mp_harness.install_stack_dump()
    a = sys.argv
    main(a[1], int(a[2]), int(a[3]), int(a[4]), a[5], int(a[6]), int(a[7]), a[8], *(a[9:11]),
         *[int(v) for v in a[11:13]])
