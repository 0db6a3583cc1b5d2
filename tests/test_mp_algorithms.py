"""Message-passing simulation (reference "MPI" mode) over the loopback transport."""
import logging

import pytest

import fedml_amd
from fedml_amd.arguments import Arguments
from fedml_amd.simulation.simulator import SimulatorMPI


def _args(opt, **kw):
    cfg = {"training_type": "simulation", "dataset": "mnist", "model": "lr", "client_num_in_total": 20,
           "client_num_per_round": 3, "comm_round": 2, "epochs": 1, "batch_size": 10, "learning_rate": 0.03,
           "frequency_of_the_test": 1, "backend": "LOOPBACK", "federated_optimizer": opt}
    cfg.update(kw)
    a = fedml_amd.init(Arguments.from_dict({"x": cfg}))
    logging.getLogger().setLevel(logging.WARNING)
    return a


@pytest.mark.parametrize("opt,kw", [
    ("FedAvg", {}),
    ("FedOpt", {"server_optimizer": "adam", "server_lr": 0.01}),
    ("FedProx", {"fedprox_mu": 0.1}),
    ("FedAvg_robust", {"defense_type": "norm_diff_clipping", "norm_bound": 1.0, "attack_freq": 1}),
    ("FedAvg_robust", {"defense_type": "weak_dp", "norm_bound": 1.0, "stddev": 0.001}),
    ("FedAvg_robust", {"defense_type": "coordinate_median"}),
])
def test_fedavg_family(opt, kw):
    a = _args(opt, **kw)
    dev, ds, m = fedml_amd._prepare(a)
    res = SimulatorMPI(a, dev, ds, m).run()
    assert len(res["history"]) >= 1
    assert res["history"][-1]["Test/Acc"] > 0.3


def test_mp_fedavg_matches_sp_fedavg():
    """Same sampling, same data, same trainer → the message-passing FedAvg global model equals the
    sequential simulator's."""
    import torch
    from fedml_amd.simulation.simulator import SimulatorSingleProcess
    a = _args("FedAvg", frequency_of_the_test=0)
    dev, ds, m = fedml_amd._prepare(a)
    import copy
    res = SimulatorMPI(a, dev, ds, copy.deepcopy(m)).run()
    b = _args("FedAvg", frequency_of_the_test=0)
    b.backend = "single_process"
    sp = SimulatorSingleProcess(b, dev, ds, copy.deepcopy(m))
    w = sp.run()
    for k in w:
        assert torch.allclose(w[k].float(), res["global_model"][k].float(), atol=1e-5), k
