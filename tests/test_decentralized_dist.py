"""Decentralized DSGD / PushSum with the workers sharded over ranks (gloo rehearsal of the RCCL path):
one all_gather of the gossip rows per iteration; params and regret equal the single-process run."""
import os
import subprocess
import sys

import mp_harness
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _run(world, out, mode):
    from test_rccl_dist import _free_port
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=os.path.dirname(HERE), OMP_NUM_THREADS="1")
    ps = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker_decentralized.py"), str(r), str(world),
                            str(port), out, mode], env=env) for r in range(world)]
    assert mp_harness.wait_all(ps, 300) == [0] * world
    return torch.load(out, weights_only=True)


@pytest.mark.parametrize("mode", ["DOL", "PUSHSUM"])
def test_sharded_gossip_equals_single_process(tmp_path, mode):
    a = _run(1, str(tmp_path / "a.pt"), mode)
    b = _run(2, str(tmp_path / "b.pt"), mode)
    assert torch.allclose(a["params"], b["params"], atol=1e-5), float((a["params"] - b["params"]).abs().max())
    assert torch.allclose(a["regret"], b["regret"], atol=1e-6)
