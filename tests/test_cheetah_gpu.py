"""Cheetah's native executor on the GPU: ResNet-56 (CIFAR-100 shape) data-parallel training through the
client-batched native HIP step (C = replicas per GPU) with the flat all-reduce of averaged gradients.

* 2 ranks × 1 replica (gloo collectives, both ranks on the box's one GPU) must equal 1 rank × 2 replicas bit for
  bit in deterministic mode — the same replicas, the same per-replica BatchNorm, the same gradient mean.
* 1 rank × 1 replica tracks plain torch fp32 SGD on the same sample order (the reference's DDP-free centralized
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


def test_native_single_replica_tracks_torch_sgd(tmp_path):
    from fedml_amd.distributed.cheetah import shard_indices
    # a small step size: batch-4 BatchNorm at lr 0.05 / momentum 0.9 is chaotic (two fp32 implementations
    # decorrelate within a few steps), which would measure the chaos, not the kernels
    got = launch(1, str(tmp_path / "n.pt"), "resnet56", replicas=1, epochs=1, env={"FEDML_TEST_LR": "0.002"},
                 timeout=300)
    assert got["native"]
    x, y, _, _ = W.data("resnet56")
    # plain fp32 on the torch side: TF32-style reduced-precision convs / GEMMs (allowed by default) alone move a
    # batch-4 BatchNorm ResNet-56's gradients by ~3 % (scripts/dbg_cheetah.py)
    torch.backends.cuda.matmul.allow_tf32 = torch.backends.cudnn.allow_tf32 = False
    model = W.make_model("resnet56").cuda()
    init = {k: v.detach().clone() for k, v in model.state_dict().items()}
    opt = torch.optim.SGD(model.parameters(), lr=0.002, momentum=0.9, weight_decay=1e-3)
    idx = shard_indices(len(x), 0, 1, 0, True, 3)
    for s in range(0, len(idx), 4):
        sel = idx[s:s + 4]
        opt.zero_grad()
        nn.functional.cross_entropy(model(x[sel].cuda()), y[sel].cuda()).backward()
        opt.step()
    num = den = 0.0
    for k, v in model.state_dict().items():
        if not v.is_floating_point() or "running" in k:
            continue
        num += float((got["state"][k].cuda() - v).norm() ** 2)
        den += float((v - init[k]).norm() ** 2)
    assert (num / den) ** 0.5 < 5e-2, (num / den) ** 0.5
