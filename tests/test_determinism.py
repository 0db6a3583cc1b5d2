"""Deterministic mode (``utils/determinism.py``): fixed RCCL algorithm/protocol, deterministic
torch algorithms, and the client-batched engine off the fp32-atomic native kernels — two runs of the RCCL
simulator give bitwise-identical global models."""
import copy
import logging
import os

import pytest
import torch

from fedml_amd.arguments import Arguments
from fedml_amd.data.synthetic import get_spec
from fedml_amd.models.cv.resnet import BasicBlock, ResNet
from fedml_amd.simulation.rccl.client_store import DeviceClientStore
from fedml_amd.simulation.rccl.simulator import RCCLSimulator


@pytest.fixture(autouse=True)
def _restore_mode():
    yield
    from fedml_amd.utils import determinism
    determinism.disable()


def _args(**kw):
    cfg = {"training_type": "simulation", "backend": "RCCL", "federated_optimizer": "FedAvg", "dataset": "cifar10",
           "model": "resnet", "client_num_in_total": 3, "client_num_per_round": 3, "comm_round": 2, "epochs": 1,
           "batch_size": 8, "client_optimizer": "sgd", "learning_rate": 0.05, "frequency_of_the_test": 0,
           "random_seed": 0, "deterministic": True}
    cfg.update(kw)
    logging.getLogger().setLevel(logging.WARNING)
    return Arguments.from_dict({"x": cfg})


def _run(dev):
    torch.manual_seed(0)
    model = ResNet(BasicBlock, [1, 1, 1], 10)
    spec = get_spec("cifar10")
    store = DeviceClientStore.synthetic_on_device(spec, [16, 16, 16], torch.device(dev), seed=0)
    sim = RCCLSimulator(_args(), torch.device(dev), None, copy.deepcopy(model), store=store)
    sim.run(2)
    out = sim.global_flat.detach().cpu().clone()
    eng = sim.engine
    sim.close()
    return out, eng


def test_deterministic_mode_env_and_reproducibility():
    from fedml_amd.utils import determinism
    a, eng = _run("cpu")
    b, _ = _run("cpu")
    assert eng.deterministic and determinism.enabled()
    assert os.environ.get("NCCL_ALGO") == "Ring" and os.environ.get("NCCL_PROTO") == "Simple"
    assert torch.are_deterministic_algorithms_enabled()
    assert torch.equal(a, b)


@pytest.mark.gpu
def test_deterministic_mode_gpu_bitwise():
    a, eng = _run("cuda")
    b, _ = _run("cuda")
    assert eng.native_step is None          # the fp32-atomic native kernels are not used in this mode
    assert torch.equal(a, b), float((a - b).abs().max())
