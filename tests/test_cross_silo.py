"""Cross-silo FL (reference `cross_silo/`): horizontal over in-process loopback, and
hierarchical with real processes — server + 2 silos × 2 data-parallel processes (TCP between
server and silo masters, gloo inside each silo)."""
import copy
import logging
import os
import subprocess
import sys
import threading

import pytest
import torch

import fedml_amd
from fedml_amd.arguments import Arguments
from fedml_amd.core.distributed.communication.transports import LoopbackRouter

HERE = os.path.dirname(os.path.abspath(__file__))


def _args(**kw):
    cfg = {"training_type": "cross_silo", "dataset": "mnist", "model": "lr", "client_num_in_total": 2,
           "client_num_per_round": 2, "comm_round": 3, "epochs": 1, "batch_size": 16, "learning_rate": 0.05,
           "frequency_of_the_test": 1, "backend": "LOOPBACK", "federated_optimizer": "FedAvg", "worker_num": 3,
           "client_id_list": "[1, 2]", "sys_perf_interval": 0, "synthetic_samples_per_client": 64}
    cfg.update(kw)
    a = Arguments.from_dict({"x": cfg})
    logging.getLogger().setLevel(logging.WARNING)
    return a


def test_horizontal_cross_silo_equals_fedavg():
    from fedml_amd.cross_silo import Client, Server
    a = _args()
    dev, ds, m = fedml_amd._prepare(fedml_amd.init(copy.copy(a)))
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
    assert "w" in out
    # same rounds with the sequential FedAvg simulator (2 of 2 clients every round ≡ data silos 0,1)
    from fedml_amd.simulation.simulator import SimulatorSingleProcess
    b = _args(backend="single_process", training_type="simulation")
    w_sp = SimulatorSingleProcess(fedml_amd.init(b), dev, ds, copy.deepcopy(m)).run()
    for k in w_sp:
        assert torch.allclose(w_sp[k].float(), out["w"][k].float(), atol=1e-5), k


@pytest.mark.slow
def test_hierarchical_cross_silo_processes(tmp_path):
    from test_rccl_dist import _free_port
    base = _free_port()
    pg1, pg2 = _free_port(), _free_port()
    out = str(tmp_path / "global.pt")
    env = dict(os.environ, PYTHONPATH=os.path.dirname(HERE), OMP_NUM_THREADS="1", FEDML_TCP_BASE_PORT=str(base))
    w = os.path.join(HERE, "dist_worker_cross_silo.py")
    cmds = [[sys.executable, w, "server", "0", "0", "0", out]]
    for silo, port in ((1, pg1), (2, pg2)):
        for r in range(2):
            cmds.append([sys.executable, w, "silo", str(silo), str(r), str(port), out])
    ps = [subprocess.Popen(c, env=env) for c in cmds]
    codes = [p.wait(timeout=300) for p in ps]
    assert codes == [0] * len(cmds), codes
    g = torch.load(out, weights_only=True)
    assert all(torch.isfinite(v.float()).all() for v in g.values())
