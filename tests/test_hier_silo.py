"""BASELINE config 5 shape on CPU processes: hierarchical cross-silo FedAvg where every silo trains
``silo_local_clients`` local clients per round on the client-batched engine, client-parallel over the
silo's 2 processes (gloo process group inside the silo, TCP between the server and the silo masters).
Reference roles: ``cross_silo/hierarchical/fedml_hierarchical_api.py:169-255``,
``client_master_manager.py:239-249``, ``trainer_dist_adapter.py:56-66``. The server's FedAvg over
silos must equal the flat RCCL simulator's FedAvg over all the silos' local clients."""
import copy
import logging
import os
import subprocess
import sys

import mp_harness
import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def _flat_reference(n_silos, n_local, rounds):
    import fedml_amd
    from fedml_amd.arguments import Arguments
    from fedml_amd.cross_silo.hierarchical.silo_batched import split_local_clients
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.simulator import RCCLSimulator
    cfg = {"training_type": "cross_silo", "scenario": "hierarchical", "dataset": "mnist", "model": "lr",
           "client_num_in_total": n_silos, "client_num_per_round": n_silos, "comm_round": rounds, "epochs": 1,
           "batch_size": 8, "learning_rate": 0.05, "frequency_of_the_test": 0, "backend": "TCP",
           "federated_optimizer": "FedAvg", "worker_num": n_silos + 1, "sys_perf_interval": 0,
           "synthetic_samples_per_client": 48, "shuffle": False, "using_gpu": False}
    args = fedml_amd.init(Arguments.from_dict({"x": cfg}))
    logging.getLogger().setLevel(logging.WARNING)
    dev, ds, m = fedml_amd._prepare(args)
    xs, ys, offs, counts, base = [], [], [], [], 0
    for s in range(n_silos):
        cd = ds[5][s]
        o, c = split_local_clients(cd, n_local)
        xs.append(cd.x)
        ys.append(cd.y)
        offs += [base + v for v in o]
        counts += c
        base += len(cd.x)
    store = DeviceClientStore(torch.cat(xs), torch.cat(ys), offs, counts)
    a = copy.copy(args)
    a.client_num_in_total = a.client_num_per_round = n_silos * n_local
    sim = RCCLSimulator(a, torch.device("cpu"), None, m, store=store)
    init = sim.global_model_state()
    sim.run(rounds)
    return sim.global_model_state(), init


@pytest.mark.slow
def test_batched_silos_equal_flat_simulator(tmp_path):
    from test_rccl_dist import _free_port
    n_silos, n_proc, n_local, rounds = 2, 2, 4, 2
    base = _free_port()
    out = str(tmp_path / "global.pt")
    env = dict(os.environ, PYTHONPATH=os.path.dirname(HERE), OMP_NUM_THREADS="1", FEDML_TCP_BASE_PORT=str(base))
    w = os.path.join(HERE, "dist_worker_hier_silo.py")
    common = [out, str(n_proc), str(n_local), "cpu", "lr", "mnist", str(rounds), str(n_silos)]
    cmds = [[sys.executable, w, "server", "0", "0", "0"] + common]
    for silo in range(1, n_silos + 1):
        port = _free_port()
        for r in range(n_proc):
            cmds.append([sys.executable, w, "silo", str(silo), str(r), str(port)] + common)
    ps = [subprocess.Popen(c, env=env) for c in cmds]
    codes = mp_harness.wait_all(ps, 300)
    assert codes == [0] * len(cmds), codes
    got = torch.load(out, weights_only=True)
    ref, init = _flat_reference(n_silos, n_local, rounds)
    assert any(not torch.allclose(ref[k].float(), init[k].float()) for k in ref)   # training moved the model
    for k in ref:
        assert torch.allclose(got[k].float(), ref[k].float(), atol=2e-6), (k, float((got[k] - ref[k]).abs().max()))
