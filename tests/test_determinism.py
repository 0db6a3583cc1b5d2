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


def _run(dev, block=BasicBlock, counts=(16, 16, 13), rounds=2, **kw):
    torch.manual_seed(0)
    model = ResNet(block, [1, 1, 1], 10)
    spec = get_spec("cifar10")
    store = DeviceClientStore.synthetic_on_device(spec, list(counts), torch.device(dev), seed=0)
    kw.setdefault("client_num_in_total", len(counts))
    kw.setdefault("client_num_per_round", len(counts))
    sim = RCCLSimulator(_args(**kw), torch.device(dev), None, copy.deepcopy(model), store=store)
    sim.run(rounds)
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
    # two rounds of small-batch BN training amplify last-bit differences (the regular mode's fp32 atomics, the
    # deterministic mode's fixed batch geometry) through ReLU-mask flips: measured 3.9e-3 / 7.5e-3 on the driver
    # box. This is a gross-error check; the deterministic step's exactness is bounded tightly against fp64 with
    # its own masks in test_native_resnet_fp32_gpu.py::test_native_step_f32_matches_reference.
    assert float((a - c).norm() / c.norm()) < 5e-2


@pytest.mark.gpu
def test_deterministic_native_step_many_geometries():
    """The native step in deterministic mode over six batch geometries (N = 8..3): the accumulation targets are
    shared across geometries, so the 16-target fixed-point registry never overflows; each geometry
    is bitwise reproducible."""
    from fedml_amd.core.arena import ParamLayout
    from fedml_amd.parallel.native_resnet import NativeResNetStep
    torch.manual_seed(0)
    model = ResNet(Bottleneck, [1, 1, 1], 10)
    layout = ParamLayout.from_module(model)
    C = 3
    flat = layout.flatten(model.state_dict()).cuda()
    def run():
        torch.manual_seed(1)
        step = NativeResNetStep(model, layout, C, "cuda")
        step.enable_deterministic()
        outs = []
        arena = flat.view(1, -1).repeat(C, 1).contiguous()     # one engine's arenas (their shape has no N)
        garena = torch.zeros_like(arena)
        try:
            for N in (8, 7, 6, 5, 4, 3):      # the step's BN pivots carry over: the sequence is the unit
                x = torch.randn(C, N, 3, 16, 16, device="cuda")
                y = torch.randint(0, 10, (C, N), device="cuda")
                rs = torch.full((C, N), 1.0 / N, device="cuda")
                arena.copy_(flat.view(1, -1).expand(C, -1))
                garena.zero_()
                step.step(arena, garena, x, y, rs, torch.ones(C, device="cuda"))
                outs.append(garena.clone())
            assert len(step._states) == 6 and len(step.det.targets) <= 8, len(step.det.targets)
            assert not step.det.poisoned()
        finally:
            step.close()
        return outs

    for ga, gb in zip(run(), run()):
        assert torch.isfinite(ga).all() and torch.equal(ga, gb)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["distilbert", "vit"])
def test_deterministic_mode_fp32_transformer_bitwise(kind):
    """fp32 transformers on the client-batched tf_f32 kernels in deterministic mode: their LN
    dgamma/dbeta and bias-gradient reductions leave the fp32 atomics for fixed-order column sums, so two
    runs of several local steps (dropout ON, keyed by seed) are bitwise identical."""
    from fedml_amd.arguments import Arguments
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    from fedml_amd.models.transformer.distilbert import distilbert
    from fedml_amd.models.transformer.vit import vit_tiny

    def run():
        torch.manual_seed(0)
        m = distilbert(3, vocab=211, dim=128, n_layers=2, n_heads=2, hidden=256, max_pos=64) \
            if kind == "distilbert" else vit_tiny(num_classes=7, img_size=32, patch=4, depth=2)
        C, n = 3, 24
        g = torch.Generator().manual_seed(1)
        if kind == "distilbert":
            x = torch.randint(1, 211, (C * n, 48), generator=g)
            y = torch.randint(0, 3, (C * n,), generator=g)
        else:
            x = torch.randn(C * n, 3, 32, 32, generator=g)
            y = torch.randint(0, 7, (C * n,), generator=g)
        args = _args(client_optimizer="adam", learning_rate=1e-3)
        eng = ClientBatchEngine(m.to("cuda"), C, "cuda", args, compute_dtype=None)
        assert eng.tf is not None and eng.deterministic
        eng.load_global(eng.layout.flatten(m.state_dict(), device="cuda"))
        store = DeviceClientStore(x.cuda(), y.cuda(), [0, n, 2 * n], [n, n, n - 5])
        eng.train(store, torch.arange(C, device="cuda"), 1, 8, 1e-3, shuffle=True, rng_key=7)
        torch.cuda.synchronize()
        out = eng.params.clone()
        eng.close()
        return out

    a, b = run(), run()
    assert torch.isfinite(a).all()
    assert torch.equal(a, b), float((a - b).abs().max())
