"""FlatDDP (bucketed, backward-overlapped all-reduce + fused flat optimizer) equals
single-process full-batch SGD with momentum (gloo, 2 ranks)."""
import os
import subprocess
import sys

import mp_harness
import pytest
import torch
import torch.nn as nn

from test_rccl_dist import _free_port

HERE = os.path.dirname(os.path.abspath(__file__))


def _run_ddp(tmp_path, mode, device="cpu"):
    out = str(tmp_path / "ddp.pt")
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=os.path.dirname(HERE), OMP_NUM_THREADS="1", FEDML_TEST_DEVICE=device)
    ps = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker_ddp.py"), str(r), "2", str(port), out, mode],
                           env=env) for r in range(2)]
    assert mp_harness.wait_all(ps, 300) == [0, 0]
    return torch.load(out, weights_only=True)


def _reference():
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(12, 32), nn.ReLU(), nn.Linear(32, 32), nn.ReLU(), nn.Linear(32, 5))
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9)
    g = torch.Generator().manual_seed(1)
    X = torch.randn(32, 12, generator=g)
    Y = torch.randint(0, 5, (32,), generator=g)
    for step in range(3):
        x, y = X.view(4, 8, 12)[step % 4], Y.view(4, 8)[step % 4]
        opt.zero_grad()
        nn.functional.cross_entropy(model(x), y).backward()
        opt.step()
    return model.state_dict()


@pytest.mark.parametrize("mode", ["flat", "torch_optim"])
def test_flat_ddp_matches_full_batch(tmp_path, mode):
    got = _run_ddp(tmp_path, mode)
    for k, v in _reference().items():
        assert torch.allclose(v, got[k], atol=1e-5), k


@pytest.mark.gpu
def test_flat_ddp_on_gpu_matches_full_batch(tmp_path):
    """Two ranks sharing the box's GPU (gloo collectives): bucket hooks, the comm stream and the
    fused flat optimizer kernel on HIP give the full-batch result."""
    got = _run_ddp(tmp_path, "flat", device="cuda")
    for k, v in _reference().items():
        assert torch.allclose(v, got[k], atol=1e-4), k
