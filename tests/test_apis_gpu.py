"""The reference-style entry points on the GPU (``using_gpu: true``): single-process simulators
(FedAvg, FedOpt, S-FedAvg Shapley valuation), the RCCL simulator through ``run_simulation``-style
setup, cross-silo horizontal over the loopback transport, and the centralized trainer."""
import copy
import logging
import threading

import pytest
import torch

import fedml_amd
from fedml_amd.arguments import Arguments

pytestmark = pytest.mark.gpu


def _args(**kw):
    cfg = {"training_type": "simulation", "dataset": "femnist", "model": "cnn", "client_num_in_total": 4,
           "client_num_per_round": 4, "comm_round": 2, "epochs": 1, "batch_size": 16, "learning_rate": 0.05,
           "frequency_of_the_test": 1, "backend": "single_process", "federated_optimizer": "FedAvg",
           "synthetic_samples_per_client": 32, "using_gpu": True, "gpu_id": 0}
    cfg.update(kw)
    a = fedml_amd.init(Arguments.from_dict({"x": cfg}))
    logging.getLogger().setLevel(logging.WARNING)
    return a


@pytest.mark.parametrize("opt,kw", [("FedAvg", {}), ("FedOpt", {"server_optimizer": "adam", "server_lr": 0.01}),
                                    ("FedProx", {"fedprox_mu": 0.1})])
def test_sp_simulator_on_gpu(opt, kw):
    from fedml_amd.simulation.simulator import SimulatorSingleProcess
    a = _args(federated_optimizer=opt, **kw)
    dev, ds, m = fedml_amd._prepare(a)
    assert dev.type == "cuda"
    w = SimulatorSingleProcess(a, dev, ds, m).run()
    assert all(torch.isfinite(v.float()).all() for v in w.values())


def test_rccl_simulator_on_gpu():
    from fedml_amd.simulation.simulator import SimulatorRCCL
    a = _args(backend="RCCL", compute_dtype="bf16")
    dev, ds, m = fedml_amd._prepare(a)
    w = SimulatorRCCL(a, dev, ds, m).run()
    assert all(torch.isfinite(v.float()).all() for v in w.values())


def test_cross_silo_loopback_on_gpu():
    from fedml_amd.core.distributed.communication.transports import LoopbackRouter
    from fedml_amd.cross_silo import Client, Server
    a = _args(training_type="cross_silo", backend="LOOPBACK", client_num_in_total=2, client_num_per_round=2,
              worker_num=3, client_id_list="[1, 2]", sys_perf_interval=0)
    dev, ds, m = fedml_amd._prepare(a)
    router = LoopbackRouter(3)
    out = {}

    def srv():
        out["w"] = Server(copy.copy(a), dev, ds, copy.deepcopy(m), comm=router).run()

    def cli(rank):
        b = copy.copy(a)
        b.rank = rank
        Client(b, dev, ds, copy.deepcopy(m), comm=router).run()

    ts = [threading.Thread(target=srv)] + [threading.Thread(target=cli, args=(r,)) for r in (1, 2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert "w" in out and all(torch.isfinite(v.float()).all() for v in out["w"].values())
