"""Hierarchical FL on the virtual-client engine (``rccl/hierarchical.py``) reproduces the sequential SP trainer
(``sp/hierarchical_fl``, reference ``single_process/hierarchical_fl``) global epoch by global epoch: full-batch
local steps make both independent of data order, so the evaluated metrics at every global epoch and the final
global model agree. Plus the reference CI invariant: one group, one group round, full batch ≡ centralized GD."""
import copy
import logging

import numpy as np
import torch

import fedml_amd
from fedml_amd.arguments import Arguments
from fedml_amd.data.data_loader import load, merge_to_centralized


def _args(**kw):
    cfg = {"training_type": "simulation", "backend": "sp", "federated_optimizer": "HierarchicalFL",
           "dataset": "mnist", "model": "lr", "client_num_in_total": 8, "client_num_per_round": 6,
           "global_comm_round": 2, "comm_round": 2, "group_comm_round": 2, "group_num": 3, "group_method": "random",
           "epochs": 2, "batch_size": 10 ** 7, "client_optimizer": "sgd", "learning_rate": 0.1,
           "frequency_of_the_test": 1, "random_seed": 0, "partition_method": "hetero", "partition_alpha": 0.5,
           "synthetic_data": True, "synthetic_train_num": 1600, "synthetic_test_num": 400, "shuffle": False}
    cfg.update(kw)
    logging.getLogger().setLevel(logging.WARNING)
    return Arguments.from_dict({"x": cfg})


def _flat(sd):
    return torch.cat([v.detach().float().reshape(-1) for _, v in sorted(sd.items())])


def _both(args):
    from fedml_amd.simulation.rccl.hierarchical import HierarchicalRCCLSimulator
    from fedml_amd.simulation.sp.hierarchical_fl.trainer import HierarchicalTrainer
    dataset, k = load(args)
    torch.manual_seed(0)
    model = fedml_amd.models.create(args, k)
    np.random.seed(123)
    sp = HierarchicalTrainer(args, torch.device("cpu"), dataset, copy.deepcopy(model))
    w_sp = sp.train()
    np.random.seed(123)
    sim = HierarchicalRCCLSimulator(args, torch.device("cpu"), dataset, copy.deepcopy(model))
    assert (sim.group_indexes == sp.group_indexes).all()
    w_rc = sim.run()
    return sp, w_sp, sim, w_rc, dataset, model


def test_hierarchical_engine_matches_sp_per_global_epoch():
    sp, w_sp, sim, w_rc, _, _ = _both(_args())
    assert torch.allclose(_flat(w_sp), _flat(w_rc), atol=2e-6), float((_flat(w_sp) - _flat(w_rc)).abs().max())
    assert len(sp.history) == len(sim.hier_history) == 2 * 2 * 2
    for a, b in zip(sp.history, sim.hier_history):
        assert a["global_epoch"] == b["global_epoch"]
        for k in ("Train/Acc", "Test/Acc"):
            assert abs(a[k] - b[k]) < 1e-6, (a["global_epoch"], k, a[k], b[k])
        for k in ("Train/Loss", "Test/Loss"):
            assert abs(a[k] - b[k]) < 1e-4 * max(1.0, abs(a[k])), (k, a[k], b[k])


def test_one_group_full_batch_equals_centralized():
    from fedml_amd.simulation.rccl.hierarchical import HierarchicalRCCLSimulator
    from fedml_amd.simulation.sp.fedavg.fedavg_api import FedAvgAPI
    args = _args(group_num=1, group_comm_round=1, epochs=1, client_num_per_round=8, global_comm_round=3,
                 comm_round=3, frequency_of_the_test=100)
    dataset, k = load(args)
    torch.manual_seed(0)
    model = fedml_amd.models.create(args, k)
    sim = HierarchicalRCCLSimulator(args, torch.device("cpu"), dataset, copy.deepcopy(model))
    w = sim.run()
    cen_args = _args(federated_optimizer="FedAvg", client_num_in_total=1, client_num_per_round=1, comm_round=3, epochs=1,
                     frequency_of_the_test=100)
    cen = FedAvgAPI(cen_args, torch.device("cpu"), merge_to_centralized(dataset), copy.deepcopy(model)).train()
    assert torch.allclose(_flat(w), _flat(cen), atol=2e-6), float((_flat(w) - _flat(cen)).abs().max())
