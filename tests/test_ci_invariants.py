"""The reference's CI invariants (``ci/CI-script-fedavg.sh``), as tests:

1. full batch, 1 local epoch: FedAvg over ALL clients ≡ centralized training on the union of their
   data (one GD step per round either way: Σ_c n_c/N·(w − η∇L_c) = w − η∇L), for the SP simulator
   and the client-batched RCCL simulator;
2. LEAF Shakespeare: 80-character strings map through the character vocabulary
   (``data/shakespeare/language_utils.py``) and the next-character RNN trains on them."""
import copy
import json
import logging

import torch

import fedml_amd
from fedml_amd.arguments import Arguments
from fedml_amd.data.data_loader import load, merge_to_centralized


def _args(**kw):
    cfg = {"training_type": "simulation", "backend": "sp", "federated_optimizer": "FedAvg", "dataset": "mnist",
           "model": "lr", "client_num_in_total": 10, "client_num_per_round": 10, "comm_round": 4, "epochs": 1,
           "batch_size": 10 ** 7, "client_optimizer": "sgd", "learning_rate": 0.03, "frequency_of_the_test": 0,
           "random_seed": 0, "partition_method": "hetero", "partition_alpha": 0.5, "synthetic_data": True,
           "synthetic_train_num": 3000, "synthetic_test_num": 500, "shuffle": False}
    cfg.update(kw)
    logging.getLogger().setLevel(logging.WARNING)
    return Arguments.from_dict({"x": cfg})


def _flat(sd):
    return torch.cat([v.detach().float().reshape(-1) for _, v in sorted(sd.items())])


def test_fedavg_full_batch_equals_centralized():
    from fedml_amd.simulation.sp.fedavg.fedavg_api import FedAvgAPI
    from fedml_amd.simulation.rccl.simulator import RCCLSimulator
    args = _args()
    dataset, k = load(args)
    torch.manual_seed(0)
    model = fedml_amd.models.create(args, k)
    counts = [dataset[4][c] for c in range(10)]
    assert len(set(counts)) > 1                                  # hetero: unequal client sizes
    fed = FedAvgAPI(args, torch.device("cpu"), dataset, copy.deepcopy(model)).train()
    cen_args = _args(client_num_in_total=1, client_num_per_round=1)
    cen = FedAvgAPI(cen_args, torch.device("cpu"), merge_to_centralized(dataset), copy.deepcopy(model)).train()
    assert torch.allclose(_flat(fed), _flat(cen), atol=2e-6), float((_flat(fed) - _flat(cen)).abs().max())
    # the RCCL simulator (client-batched engine, on-device weighted sum) holds the same invariant
    rargs = _args(backend="RCCL")
    sim = RCCLSimulator(rargs, torch.device("cpu"), dataset, copy.deepcopy(model))
    sim.run(int(rargs.comm_round))
    got = _flat(sim.global_model_state())
    assert torch.allclose(got, _flat(cen), atol=2e-6), float((got - _flat(cen)).abs().max())


def _write_leaf(root, users, n, rng):
    from fedml_amd.data.shakespeare import ALL_LETTERS
    for split in ("train", "test"):
        (root / split).mkdir(parents=True)
        data = {"users": users, "num_samples": [n] * len(users), "user_data": {}}
        for u in users:
            xs, ys = [], []
            for _ in range(n):
                s = "".join(ALL_LETTERS[i] for i in rng.integers(0, len(ALL_LETTERS), 81))
                xs.append(s[:80])
                ys.append(s[80])
            data["user_data"][u] = {"x": xs, "y": ys}
        (root / split / "all_data.json").write_text(json.dumps(data))


def test_leaf_shakespeare_character_pipeline(tmp_path):
    import numpy as np
    from fedml_amd.data.shakespeare import ALL_LETTERS, VOCAB_SIZE, letter_to_index, word_to_indices
    from fedml_amd.simulation.sp.fedavg.fedavg_api import FedAvgAPI
    assert VOCAB_SIZE == 90 and len(ALL_LETTERS) == 86
    assert word_to_indices("dh l") == [0, 1, 13, 2]
    assert letter_to_index("é") == len(ALL_LETTERS)       # unknown → OOV id (embeddable)
    _write_leaf(tmp_path, ["u0", "u1", "u2"], 12, np.random.default_rng(0))
    args = _args(dataset="shakespeare", model="rnn", client_num_in_total=3, client_num_per_round=3,
                 synthetic_data=False, data_cache_dir=str(tmp_path), batch_size=4, comm_round=1, learning_rate=0.8)
    dataset, k = load(args)
    assert int(args.client_num_in_total) == 3
    cd = dataset[5][0]
    assert cd.x.dtype == torch.int64 and tuple(cd.x.shape) == (12, 80) and cd.y.dtype == torch.int64
    raw = json.loads((tmp_path / "train" / "all_data.json").read_text())["user_data"]["u0"]
    assert sorted(cd.y.tolist()) == sorted(letter_to_index(c) for c in raw["y"])   # same samples (shuffled)
    model = fedml_amd.models.create(args, k)
    w = FedAvgAPI(args, torch.device("cpu"), dataset, model).train()
    assert all(torch.isfinite(v).all() for v in w.values() if v.is_floating_point())
