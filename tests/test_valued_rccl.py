"""S-FedAvg / HS-FedAvg on the RCCL virtual-client engine (``simulation/rccl/valued.py``) against the sequential SP
simulator (the reference's loop: one client after another, class-balanced CE, clip 1.0): the batched path must
reproduce the SP run's sampled-client sequence, φ and Shapley values round by round (LR / MNIST-shaped data,
CPU) — and the 2-rank gloo run (sharded coalition evaluation) must reproduce the 1-rank run."""
import copy
import logging
import os
import subprocess
import sys

import mp_harness
import numpy as np
import pytest
import torch

import fedml_amd
from fedml_amd.arguments import Arguments

HERE = os.path.dirname(os.path.abspath(__file__))


def _setup(opt, **kw):
    cfg = {"training_type": "simulation", "dataset": "mnist", "model": "lr", "client_num_in_total": 8,
           "client_num_per_round": 4, "comm_round": 3, "epochs": 1, "batch_size": 16, "learning_rate": 0.1,
           "frequency_of_the_test": 0, "backend": "single_process", "federated_optimizer": opt,
           "synthetic_train_samples_per_client": 64, "partition_method": "hetero", "valid_samples": 200,
           "shuffle": False, "random_seed": 0}
    cfg.update(kw)
    a = fedml_amd.init(Arguments.from_dict({"x": cfg}))
    logging.getLogger().setLevel(logging.WARNING)
    dev, ds, m = fedml_amd._prepare(a)
    for cd in ds[5].values():          # both simulators walk every client's samples in stored order
        cd.shuffle = False
    return a, dev, ds, m


def _sp(opt, **kw):
    from fedml_amd.simulation.simulator import SimulatorSingleProcess
    a, dev, ds, m = _setup(opt, **kw)
    np.random.seed(0)
    sim = SimulatorSingleProcess(a, dev, ds, m)
    sampled = []
    orig = sim.fl_trainer._client_sampling
    sim.fl_trainer._client_sampling = lambda *x, **k: sampled.append(orig(*x, **k)) or sampled[-1]
    w = sim.run()
    return sim.fl_trainer.results, sampled, w


def _rccl(opt, **kw):
    from fedml_amd.simulation.rccl.valued import ValuedRCCLSimulator
    a, dev, ds, m = _setup(opt, **kw)
    np.random.seed(0)
    sim = ValuedRCCLSimulator(a, dev, ds, m)
    w = sim.run()
    sim.close()
    return sim.results, w


@pytest.mark.parametrize("opt,kw", [("S-FedAvg", {}), ("S-FedAvg", {"sv_approaching": True}),
                                    ("HS-FedAvg", {"dataset": "cifar10", "model": "lr",
                                                   "synthetic_train_samples_per_client": 24, "valid_samples": 64})])
def test_valued_rccl_reproduces_sp(opt, kw):
    sp, sampled, w_sp = _sp(opt, **kw)
    rc, w_rc = _rccl(opt, **kw)
    for r in range(3):
        assert rc["sampled"][r] == [int(c) for c in sampled[r]], r
        np.testing.assert_allclose(rc["phi"][r], sp["phi"][r], atol=2e-3, rtol=0)
        np.testing.assert_allclose(rc["sv"][r], sp["sv"][r], atol=2e-3, rtol=0)
    for k, v in w_sp.items():
        if v.is_floating_point():
            assert torch.allclose(w_rc[k].float(), v.float(), atol=2e-4, rtol=1e-3), k
    assert any(abs(p - 1 / 8) > 1e-6 for p in rc["phi"][2])


def test_class_weight_table_matches_reference_formula():
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.valued import class_weight_table
    from fedml_amd.simulation.sp.valuation_base import calc_class_weight
    y = torch.tensor([0, 0, 1, 3, 3, 3, 2, 2, 0])
    store = DeviceClientStore(torch.zeros(9, 2), y, [0, 6], [6, 3])
    t = class_weight_table(store, 5)
    for c, (lo, n) in enumerate([(0, 6), (6, 3)]):
        ref = calc_class_weight([(None, y[lo:lo + n])], 5)
        assert torch.allclose(t[c], ref), (t[c], ref)


def test_valued_rccl_two_ranks_equal_one_rank(tmp_path):
    """Sharded coalition evaluation + all-gathered client models: 2 gloo ranks reproduce 1 rank."""
    outs = []
    for world in (1, 2):
        out = str(tmp_path / f"v{world}.pt")
        port = mp_harness.free_port()
        env = dict(os.environ, PYTHONPATH=os.path.dirname(HERE), OMP_NUM_THREADS="1")
        ps = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker_valued.py"), str(r), str(world),
                                str(port), out], env=env) for r in range(world)]
        assert mp_harness.wait_all(ps, 300) == [0] * world
        outs.append(torch.load(out, weights_only=True))
    a, b = outs
    assert a["sampled"] == b["sampled"]
    for r in a["phi"]:
        np.testing.assert_allclose(a["phi"][r], b["phi"][r], atol=1e-5, rtol=0)
    assert float((a["w"] - b["w"]).norm() / a["w"].norm()) < 1e-5
