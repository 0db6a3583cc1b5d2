"""FedNova on the client-batched RCCL simulator (normalised averaging + server momentum through the fused
K11 kernel / its CPU reference) against the sequential FedNova of the SP simulator (reference
``single_process/fednova/fednova_trainer.py``): unequal client sizes (LDA partition) give unequal local step
counts, which is exactly where FedNova departs from FedAvg."""
import copy
import logging

import pytest
import torch

import fedml_amd
from fedml_amd.arguments import Arguments
from fedml_amd.data.data_loader import load


def _args(**kw):
    cfg = {"training_type": "simulation", "backend": "sp", "federated_optimizer": "FedNova", "dataset": "mnist",
           "model": "lr", "client_num_in_total": 6, "client_num_per_round": 6, "comm_round": 3, "epochs": 1,
           "batch_size": 16, "client_optimizer": "sgd", "learning_rate": 0.05, "frequency_of_the_test": 0,
           "random_seed": 0, "partition_method": "hetero", "partition_alpha": 0.5, "synthetic_data": True,
           "synthetic_train_num": 600, "synthetic_test_num": 100, "shuffle": False}
    cfg.update(kw)
    logging.getLogger().setLevel(logging.WARNING)
    return Arguments.from_dict({"x": cfg})


def _flat(sd):
    return torch.cat([v.detach().float().reshape(-1) for k, v in sorted(sd.items()) if v.is_floating_point()])


@pytest.mark.parametrize("kw", [{}, {"momentum": 0.9}, {"gmf": 0.5}, {"mu": 0.01}])
def test_fednova_rccl_equals_sp(kw):
    from fedml_amd.simulation.rccl.simulator import RCCLSimulator
    from fedml_amd.simulation.sp.fednova.fednova_api import FedNovaAPI
    args = _args(**kw)
    dataset, k = load(args)
    counts = [dataset[4][c] for c in range(6)]
    assert len({(n + 15) // 16 for n in counts}) > 1            # unequal local step counts
    torch.manual_seed(0)
    model = fedml_amd.models.create(args, k)
    ref = FedNovaAPI(args, torch.device("cpu"), dataset, copy.deepcopy(model)).train()
    rargs = _args(backend="RCCL", **kw)
    sim = RCCLSimulator(rargs, torch.device("cpu"), dataset, copy.deepcopy(model))
    assert sim.fednova
    sim.run(int(rargs.comm_round))
    got = _flat(sim.global_model_state())
    assert torch.allclose(got, _flat(ref), atol=1e-5), float((got - _flat(ref)).abs().max())
    fedavg = RCCLSimulator(_args(backend="RCCL", federated_optimizer="FedAvg", **kw), torch.device("cpu"), dataset,
                           copy.deepcopy(model))
    fedavg.run(int(rargs.comm_round))
    assert not torch.allclose(_flat(fedavg.global_model_state()), got, atol=1e-4)   # FedNova ≠ FedAvg here


def test_fednova_normalizer_matches_local_optimizer():
    """The host-side a_i / τ_eff of the RCCL path equals the counters of the FedNova local optimizer."""
    from fedml_amd.simulation.rccl.simulator import fednova_normalizer
    from fedml_amd.trainers.fednova import FedNovaOptimizer
    for mom, mu in [(0.0, 0.0), (0.9, 0.0), (0.0, 0.1), (0.5, 0.1)]:
        p = torch.nn.Parameter(torch.zeros(3))
        opt = FedNovaOptimizer([p], lr=0.1, momentum=mom, mu=mu)
        for _ in range(7):
            p.grad = torch.ones(3)
            opt.step()
        a, t = fednova_normalizer(7, 0.1, mom, mu)
        assert abs(a - opt.local_normalizing_vec) < 1e-9 and abs(t - opt.tau_eff()) < 1e-9, (mom, mu)
