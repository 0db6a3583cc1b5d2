"""The RCCL simulator's evaluation reports the fork's per-round metrics (reference
`single_process/fedavg/fedavg_api.py:130-177,238-326`, `my_model_trainer_classification.py:113-154`) and matches
the SP simulator's record round by round: with full-batch local steps both simulators hold the same global model
(``test_ci_invariants``), so every metric — federation scalars, per-client accuracy lists, per-class recall /
precision dicts, Global/Acc / Loss / Recall of the target label — must agree."""
import copy
import logging

import numpy as np
import pytest
import torch

import fedml_amd
from fedml_amd.arguments import Arguments
from fedml_amd.data.data_loader import load


def _args(**kw):
    cfg = {"training_type": "simulation", "backend": "sp", "federated_optimizer": "FedAvg", "dataset": "mnist",
           "model": "lr", "client_num_in_total": 6, "client_num_per_round": 6, "comm_round": 3, "epochs": 1,
           "batch_size": 10 ** 7, "client_optimizer": "sgd", "learning_rate": 0.1, "frequency_of_the_test": 1,
           "random_seed": 0, "partition_method": "hetero", "partition_alpha": 0.5, "synthetic_data": True,
           "synthetic_train_num": 1200, "synthetic_test_num": 300, "shuffle": False, "target_label": 3}
    cfg.update(kw)
    logging.getLogger().setLevel(logging.WARNING)
    return Arguments.from_dict({"x": cfg})


def _close(a, b, tol=1e-5):
    if isinstance(a, dict):
        assert set(a) == set(b), (a, b)
        for k in a:
            _close(a[k], b[k], tol)
    elif isinstance(a, (list, tuple)):
        assert len(a) == len(b)
        for u, v in zip(a, b):
            _close(u, v, tol)
    elif a is None:
        assert b is None
    else:
        assert abs(float(a) - float(b)) <= tol * max(1.0, abs(float(a))), (a, b)


def test_rccl_metrics_match_sp_record():
    from fedml_amd.simulation.rccl.simulator import RCCLSimulator
    from fedml_amd.simulation.sp.fedavg.fedavg_api import FedAvgAPI
    args = _args()
    dataset, k = load(args)
    torch.manual_seed(0)
    model = fedml_amd.models.create(args, k)
    sp = FedAvgAPI(args, torch.device("cpu"), dataset, copy.deepcopy(model))
    sp.train()
    rargs = _args(backend="RCCL")
    sim = RCCLSimulator(rargs, torch.device("cpu"), dataset, copy.deepcopy(model))
    sim.run(int(rargs.comm_round))
    keys = ["Train/Acc", "Train/Loss", "Test/Acc", "Test/Loss", "Authority/Train/Acc", "Authority/Test/Acc",
            "Train/AccPerClient", "Test/AccPerClient", "Test/Recall", "Test/Precision", "Global/Acc", "Global/Loss",
            "Global/Recall"]
    for r in range(int(args.comm_round)):
        a, b = sp.res_dict[r], sim.history[r]
        for key in keys:
            assert key in a and key in b, (r, key)
            _close(a[key], b[key], 1e-4 if "Loss" in key else 1e-6)
        assert len(b["Test/Recall"]) == 6 and all(isinstance(d, dict) for d in b["Test/Recall"])
        assert b["Global/Recall"] is not None
    # learning: the federation's train accuracy rises over the rounds
    assert sim.history[2]["Train/Acc"] > sim.history[0]["Train/Acc"]


def test_class_rates_fork_formula():
    from fedml_amd.simulation.common import class_rates
    # class 0: 2 of 3 right; class 1: present, never right, predicted twice; class 2: absent from the labels
    rec, prec = class_rates([2, 0, 0], [3, 1, 0], [2, 2, 0])
    assert set(rec) == {0, 1} and set(prec) == {0, 1}
    assert rec[0] == pytest.approx(2 / 3) and rec[1] == 0.0
    assert prec[0] == pytest.approx(1.0) and prec[1] == 0.0
    # a present class that was never predicted: (0 + 1e-13) / (0 + 1e-13) = 1 (the fork's smoothing)
    _, prec = class_rates([0], [4], [0])
    assert prec[0] == pytest.approx(1.0)


def test_eval_stats_cpu_matches_direct_counts():
    from fedml_amd import ops
    g = torch.Generator().manual_seed(0)
    z = torch.randn(257, 7, generator=g)
    y = torch.randint(0, 7, (257,), generator=g)
    y[5] = -1                                                   # padding row
    grp = torch.randint(0, 3, (257,), generator=g).to(torch.int32)
    grp[9] = -1                                                 # padding group
    sums, cls = ops.eval_stats(z, y, grp, num_groups=3, with_classes=True)
    ok = (y >= 0) & (grp >= 0)
    pred = z.argmax(1)
    ce = torch.nn.functional.cross_entropy(z, y.clamp_min(0), reduction="none")
    for c in range(3):
        m = ok & (grp == c)
        assert sums[c, 0] == float(((pred == y) & m).sum())
        assert float(sums[c, 1]) == pytest.approx(float(ce[m].sum()), rel=1e-5)
        assert sums[c, 2] == float(m.sum())
        for k in range(7):
            assert cls[c, 0, k] == int(((pred == y) & m & (y == k)).sum())
            assert cls[c, 1, k] == int((m & (y == k)).sum())
            assert cls[c, 2, k] == int((m & (pred == k)).sum())
    assert np.isfinite(sums.numpy()).all()


def test_eval_metrics_world_invariant(tmp_path):
    """The evaluation's shards (global test rows split by rank, clients c ≡ rank mod world) and its one all-reduce
    give the same per-round metric record on 1 and 2 gloo ranks (full-batch training: the same global models)."""
    import json
    import os
    import subprocess
    import sys
    import mp_harness
    here = os.path.dirname(os.path.abspath(__file__))
    out = {}
    for world in (1, 2):
        port = mp_harness.free_port()
        path = str(tmp_path / f"h{world}.json")
        env = dict(os.environ, PYTHONPATH=os.path.dirname(here), OMP_NUM_THREADS="1")
        ps = [subprocess.Popen([sys.executable, os.path.join(here, "dist_worker_eval.py"), str(r), str(world),
                                str(port), path], env=env) for r in range(world)]
        assert mp_harness.wait_all(ps, 300) == [0] * world
        out[world] = json.load(open(path))
    assert set(out[1]) == set(out[2]) and len(out[1]) == 3
    for r in out[1]:
        _close(out[1][r], out[2][r], 1e-5)
