"""Multi-process RCCL-simulator path rehearsed on CPU with gloo: the global model after N rounds
must not depend on how many ranks the clients were packed onto (the all-reduced partial sums
Σ n_c·w_c ‖ Σ n_c are order-independent up to fp32 summation)."""
import os
import socket
import subprocess
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(world, out, model, clients):
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=os.path.dirname(HERE), OMP_NUM_THREADS="2")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker_rccl_sim.py"), str(r), str(world),
                               str(port), out, model, str(clients), "3"], env=env)
             for r in range(world)]
    codes = [p.wait(timeout=600) for p in procs]
    assert codes == [0] * world, codes
    return torch.load(out, weights_only=True)


@pytest.mark.parametrize("model,clients", [("lr", 7), ("resnet_shallow", 3)])
def test_rccl_sim_world_size_invariance(tmp_path, model, clients):
    w1 = _launch(1, str(tmp_path / "w1.pt"), model, clients)
    w2 = _launch(2, str(tmp_path / "w2.pt"), model, clients)
    assert w1.shape == w2.shape
    rel = float((w1 - w2).norm() / w1.norm())
    assert rel < (1e-5 if model == "lr" else 1e-3), rel
