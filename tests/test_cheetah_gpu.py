"""Cheetah's native executor on the GPU: ResNet-56 (CIFAR-100 shape) data-parallel training through the
client-batched native HIP step (C = replicas per GPU) with the flat all-reduce of averaged gradients.

* 2 ranks × 1 replica (gloo collectives, both ranks on the box's one GPU) must equal 1 rank × 2 replicas bit for
  bit in deterministic mode — the same replicas, the same per-replica BatchNorm, the same gradient mean.
* 1 rank × 1 replica tracks fp64 SGD on the same sample order (the reference's DDP-free centralized
  trainer) within the fp32 spread."""
import os
import sys

import pytest
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import dist_worker_cheetah as W  # noqa: E402
from test_cheetah import launch  # noqa: E402

pytestmark = pytest.mark.gpu
_ENV = dict(FEDML_AMD_DIST_BACKEND="gloo", FEDML_AMD_DETERMINISTIC="1", HSA_ENABLE_IPC_MODE_LEGACY="0")


def test_native_two_ranks_equal_one_rank_two_replicas(tmp_path):
    a = launch(1, str(tmp_path / "r1.pt"), "resnet56", replicas=2, epochs=2, env=_ENV, timeout=400)
    b = launch(2, str(tmp_path / "r2.pt"), "resnet56", replicas=1, epochs=2, env=_ENV, timeout=400)
    assert a["native"] and b["native"]
    for k, v in a["state"].items():
        assert torch.equal(v, b["state"][k]), (k, float((v.float() - b["state"][k].float()).abs().max()))
    assert a["eval"]["test_acc"] == b["eval"]["test_acc"]
    assert a["samples"] == b["samples"] == 2 * 2 * 19


def _torch_epoch(x, y, idx, dev, dtype, lr):
    model = W.make_model("resnet56").to(dev, dtype)
    init = {k: v.detach().clone() for k, v in model.state_dict().items()}
    opt = torch.optim.SGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=1e-3)
    for s in range(0, len(idx), 4):
        sel = idx[s:s + 4]
        opt.zero_grad()
        nn.functional.cross_entropy(model(x[sel].to(dev, dtype)), y[sel].to(dev)).backward()
        opt.step()
    return {k: v.detach().cpu().double() for k, v in model.state_dict().items()}, init


def test_native_single_replica_tracks_torch_sgd(tmp_path):
    """One epoch of batch-4 SGD (momentum 0.9, weight decay) on the native step against the same schedule in fp64
    (CPU): the native trajectory must be at least as close to exact arithmetic as plain fp32 torch on the GPU.
    Batch-4 BatchNorm through 56 layers is ill-conditioned — one fp32 torch step is already ~2 % off fp64 in
    gradient norm (scripts/dbg_cheetah.py; the native step measured 1 %) — so torch fp32 is not the yardstick."""
    from fedml_amd.distributed.cheetah import shard_indices
    lr = 0.002
    got = launch(1, str(tmp_path / "n.pt"), "resnet56", replicas=1, epochs=1, env={"FEDML_TEST_LR": str(lr)},
                 timeout=300)
    assert got["native"]
    x, y, _, _ = W.data("resnet56")
    idx = shard_indices(len(x), 0, 1, 0, True, 3)
    torch.backends.cuda.matmul.allow_tf32 = torch.backends.cudnn.allow_tf32 = False
    ref, init = _torch_epoch(x, y, idx, "cpu", torch.float64, lr)
    t32, _ = _torch_epoch(x, y, idx, "cuda", torch.float32, lr)

    def err(sd):
        num = den = 0.0
        for k, v in ref.items():
            if not v.is_floating_point() or "running" in k:
                continue
            num += float((sd[k].double() - v).norm() ** 2)
            den += float((v - init[k].cpu().double()).norm() ** 2)
        return (num / den) ** 0.5

    e_nat, e_t32 = err(got["state"]), err(t32)
    assert e_nat < max(2.0 * e_t32, 1e-3), (e_nat, e_t32)


def test_native_transformer_dp_world_invariant(tmp_path):
    """ViT data parallelism on the native fp32 transformer kernels (replicas = client slots of the batched
    transformer executor) with backward-overlapped gradient buckets: 2 ranks × 1 replica ≡ 1 rank × 2 replicas bit
    for bit (deterministic mode), and buckets were all-reduced while the backward was still being issued (the
    kernels' completion notifications drive them)."""
    a = launch(1, str(tmp_path / "v1.pt"), "vit_gpu", replicas=2, epochs=2, env=_ENV, timeout=400)
    b = launch(2, str(tmp_path / "v2.pt"), "vit_gpu", replicas=1, epochs=2, env=_ENV, timeout=400)
    assert a["native"] and b["native"]
    diff = {k: float((v.float() - b["state"][k].float()).abs().max()) for k, v in a["state"].items()
            if not torch.equal(v, b["state"][k])}
    assert not diff, diff
    assert a["overlapped"] > 0 and b["overlapped"] > 0
