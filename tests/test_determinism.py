"""Deterministic mode (``utils/determinism.py``): fixed RCCL algorithm/protocol, deterministic
torch algorithms, and the native HIP step with its cross-workgroup fp32 atomics switched to order-independent
fixed-point accumulation (ops/det_ops.py) — two runs of the RCCL simulator give bitwise-identical global
models on the same kernels the headline uses."""
import copy
import logging
import os

import pytest
import torch

from fedml_amd.arguments import Arguments
from fedml_amd.data.synthetic import get_spec
from fedml_amd.models.cv.resnet import BasicBlock, Bottleneck, ResNet
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


def _run(dev, block=BasicBlock, **kw):
    torch.manual_seed(0)
    model = ResNet(block, [1, 1, 1], 10)
    spec = get_spec("cifar10")
    store = DeviceClientStore.synthetic_on_device(spec, [16, 16, 13], torch.device(dev), seed=0)
    sim = RCCLSimulator(_args(**kw), torch.device(dev), None, copy.deepcopy(model), store=store)
    sim.run(2)
    out = sim.global_flat.detach().cpu().clone()
    eng = sim.engine
    used_det = eng.native_step is not None and eng.native_step.det is not None
    if used_det:
        assert not eng.native_step.det.poisoned()
    sim.close()
    return out, eng, used_det


def test_deterministic_mode_env_and_reproducibility():
    from fedml_amd.utils import determinism
    a, eng, _ = _run("cpu")
    b, _, _ = _run("cpu")
    assert eng.deterministic and determinism.enabled()
    assert os.environ.get("NCCL_ALGO") == "Ring" and os.environ.get("NCCL_PROTO") == "Simple"
    assert torch.are_deterministic_algorithms_enabled()
    assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("block", [BasicBlock, Bottleneck])
def test_deterministic_mode_gpu_bitwise(block):
    """Native kernels (3×3 tile, fused 1×1 backward, generic / wide weight gradients, BN statistics) in
    deterministic mode: bitwise-identical after two rounds with a ragged last batch, and equal to the
    regular (fp32-atomic) mode to fp32 noise."""
    from fedml_amd.utils import determinism
    a, eng, used = _run("cuda", block)
    b, _, _ = _run("cuda", block)
    assert used and eng.native_step is not None     # the headline kernels, not a torch fallback
    assert torch.equal(a, b), float((a - b).abs().max())
    determinism.disable()
    c, eng2, used2 = _run("cuda", block, deterministic=False)
    assert eng2.native_step is not None and not used2
    assert float((a - c).norm() / c.norm()) < 1e-4
