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


@pytest.mark.parametrize("kw", [{}, {"momentum": 0.9}, {"gmf": 0.5}, {"mu": 0.01},
                                {"momentum": 0.5, "mu": 0.01, "wd": 0.001},
                                {"gmf": 0.5, "fednova_gmf_persist": True}])
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


def test_fednova_gmf_resets_each_round_like_reference():
    """The reference re-creates its global momentum buffer at the start of every round
    (fednova_trainer.py:80): buf = cum_grad / lr, then w −= lr·buf, i.e. w −= cum_grad — so any gmf gives
    the gmf = 0 trajectory. Pinned on both simulators; the persistent variant (opt-in) differs."""
    from fedml_amd.simulation.rccl.simulator import RCCLSimulator
    args = _args(backend="RCCL")
    dataset, k = load(args)
    torch.manual_seed(0)
    model = fedml_amd.models.create(args, k)
    out = {}
    for name, kw in {"g0": {}, "g5": {"gmf": 0.5}, "g5p": {"gmf": 0.5, "fednova_gmf_persist": True}}.items():
        sim = RCCLSimulator(_args(backend="RCCL", **kw), torch.device("cpu"), dataset, copy.deepcopy(model))
        sim.run(3)
        out[name] = _flat(sim.global_model_state())
    assert torch.allclose(out["g0"], out["g5"], atol=1e-6)
    assert not torch.allclose(out["g0"], out["g5p"], atol=1e-4)


def test_fednova_prox_enters_momentum_buffer_like_reference():
    """Reference step (fednova.py:129-142): d_p = buf after the momentum update, then d_p.add_(mu, w − w0)
    in place — the proximal term accumulates in the buffer. Hand-computed two steps."""
    from fedml_amd.trainers.fednova import FedNovaOptimizer
    p = torch.nn.Parameter(torch.tensor([1.0]))
    opt = FedNovaOptimizer([p], lr=0.1, momentum=0.5, mu=0.2)
    w0, lr, rho, mu = 1.0, 0.1, 0.5, 0.2
    g1, g2 = 2.0, 3.0
    p.grad = torch.tensor([g1]); opt.step()
    buf = g1 + mu * (1.0 - w0)
    w = 1.0 - lr * buf
    p.grad = torch.tensor([g2]); opt.step()
    buf = rho * buf + g2 + mu * (w - w0)
    w = w - lr * buf
    assert abs(float(p) - w) < 1e-6
    assert abs(float(opt.state[p]["momentum_buffer"]) - buf) < 1e-6
