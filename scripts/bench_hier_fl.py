"""Hierarchical FL (reference `single_process/hierarchical_fl`): global rounds/s of the virtual-client engine
(``rccl/hierarchical.py``) against the sequential SP trainer (``sp/hierarchical_fl``) on the same GPU, same data.

    python scripts/bench_hier_fl.py --impl rccl|sp --clients 20 --groups 4 --group-rounds 2 --rounds 2
"""
import argparse
import copy
import json
import logging
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--impl", default="rccl")
    p.add_argument("--model", default="resnet56")
    p.add_argument("--dataset", default="cifar100")
    p.add_argument("--clients", type=int, default=20)
    p.add_argument("--samples-per-client", type=int, default=500)
    p.add_argument("--groups", type=int, default=4)
    p.add_argument("--group-rounds", type=int, default=2)
    p.add_argument("--epochs", type=int, default=1)
    p.add_argument("--rounds", type=int, default=2, help="timed global rounds (after one warm-up round)")
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--lr", type=float, default=0.01)
    a = p.parse_args()
    import numpy as np
    import torch
    import fedml_amd
    from fedml_amd.arguments import Arguments
    from fedml_amd.data.data_loader import load
    logging.getLogger().setLevel(logging.WARNING)
    cfg = {"training_type": "simulation", "backend": "RCCL", "federated_optimizer": "HierarchicalFL",
           "dataset": a.dataset, "model": a.model, "client_num_in_total": a.clients, "client_num_per_round": a.clients,
           "global_comm_round": a.rounds + 1, "comm_round": a.rounds + 1, "group_comm_round": a.group_rounds,
           "group_num": a.groups, "group_method": "random", "epochs": a.epochs, "batch_size": a.batch_size,
           "client_optimizer": "sgd", "learning_rate": a.lr, "frequency_of_the_test": 10 ** 6, "random_seed": 0,
           "partition_method": "homo", "synthetic_data": True,
           "synthetic_train_num": a.clients * a.samples_per_client, "synthetic_test_num": 1000}
    args = Arguments.from_dict({"x": cfg})
    dataset, k = load(args)
    torch.manual_seed(0)
    model = fedml_amd.models.create(args, k)
    dev = torch.device("cuda:0")
    np.random.seed(123)
    if a.impl == "rccl":
        from fedml_amd.simulation.rccl.hierarchical import HierarchicalRCCLSimulator
        sim = HierarchicalRCCLSimulator(args, dev, None, copy.deepcopy(model),
                                        store=None if dataset is None else _store(dataset, dev))
        sim.run(1)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sim.run(a.rounds)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        executor = sim.engine.executor
        loss = float(sim.engine.last_loss)
    else:
        from fedml_amd.simulation.sp.hierarchical_fl.trainer import HierarchicalTrainer
        tr = HierarchicalTrainer(args, dev, dataset, copy.deepcopy(model))
        tr._local_test_on_all_clients = lambda ge: {}     # no evaluation in either timed loop
        tr.global_rounds = 1
        tr.train()
        torch.cuda.synchronize()
        tr.global_rounds = a.rounds
        t0 = time.perf_counter()
        tr.train()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        executor, loss = "sequential torch (SP)", None
    print(json.dumps({"metric": f"hierarchical FL global rounds/s ({a.model}, {a.clients} clients, {a.groups} groups, "
                                f"{a.group_rounds} group rounds x {a.epochs} epochs)",
                      "impl": a.impl, "executor": executor, "value": round(a.rounds / dt, 4), "unit": "rounds/s",
                      "s_per_round": round(dt / a.rounds, 3), "dtype": "fp32", "final_train_loss": loss,
                      "data": "synthetic cifar-shaped, random-init weights"}), flush=True)


def _store(dataset, dev):
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    return DeviceClientStore.from_client_data(dataset[5], dev)


if __name__ == "__main__":
    main()
