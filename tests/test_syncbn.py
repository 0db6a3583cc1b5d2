"""Synchronised BatchNorm over ranks (reference model/cv/batchnorm_utils.py, here process-per-GPU with one
all-reduce per layer/direction): two ranks with half a batch each produce exactly the full-batch
BatchNorm output, input gradient, parameter gradients and running statistics (gloo rehearsal)."""
import os
import subprocess
import sys

import torch

import mp_harness

HERE = os.path.dirname(os.path.abspath(__file__))


def test_syncbn_two_ranks_equal_full_batch(tmp_path):
    from test_rccl_dist import _free_port
    out = str(tmp_path / "s.pt")
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=os.path.dirname(HERE), OMP_NUM_THREADS="1")
    ps = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker_syncbn.py"), str(r), "2", str(port), out],
                           env=env) for r in range(2)]
    assert mp_harness.wait_all(ps, 120) == [0, 0]
    r = torch.load(out, weights_only=True)
    g = torch.Generator().manual_seed(0)
    x = (torch.randn(8, 6, 5, 5, generator=g) * 3 + 1).requires_grad_(True)
    dy = torch.randn(8, 6, 5, 5, generator=g)
    bn = torch.nn.BatchNorm2d(6)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5, generator=g)
        bn.bias.uniform_(-0.5, 0.5, generator=g)
    y = bn(x)
    y.backward(dy)
    n = 4 * 6 * 25
    got_y = torch.cat([p[:n].view(4, 6, 5, 5) for p in r["parts"]])
    got_dx = torch.cat([p[n:].view(4, 6, 5, 5) for p in r["parts"]])
    torch.testing.assert_close(got_y, y.detach(), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(got_dx, x.grad, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(r["wg"], bn.weight.grad, atol=1e-4, rtol=1e-5)
    torch.testing.assert_close(r["bg"], bn.bias.grad, atol=1e-4, rtol=1e-5)
    torch.testing.assert_close(r["rm"], bn.running_mean, atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(r["rv"], bn.running_var, atol=1e-5, rtol=1e-5)
