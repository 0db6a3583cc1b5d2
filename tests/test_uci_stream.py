"""UCI (SUSY-format) streaming split for decentralized online learning (reference
data/UCI/data_loader_for_susy_and_ro.py): a β fraction clustered per client, the rest streamed in order,
every client's stream exactly sample_num/n_clients long; the stacked streams drive DecentralizedFLAPI."""
import numpy as np
import torch

from fedml_amd.data.uci_stream import load_streams, stack_streams


def _csv(path, n, rng):
    with open(path, "w") as f:
        for i in range(n):
            c = i % 2
            x = rng.normal(loc=4.0 * c, size=18)
            f.write(",".join([f"{float(c):.1f}"] + [f"{v:.5f}" for v in x]) + "\n")


def test_streams_and_decentralized_run(tmp_path):
    from fedml_amd.arguments import Arguments
    from fedml_amd.models.linear.lr import LogisticRegression
    from fedml_amd.simulation.sp.decentralized.decentralized_api import DecentralizedFLAPI
    p = str(tmp_path / "SUSY.csv")
    _csv(p, 130, np.random.default_rng(0))
    s = load_streams(p, "SUSY", [0, 1, 2, 3], 120, beta=0.5)
    assert all(len(v[0]) == 30 and v[0].shape[1] == 18 for v in s.values())
    idx_all = torch.cat([v[0] for v in s.values()])
    assert len(torch.unique(idx_all, dim=0)) == 120                     # no sample used twice
    # the clustered half is label-skewed: some client's adversarial part is mostly one class
    X, Y = stack_streams(s)
    assert X.shape == (4, 30, 18) and Y.shape == (4, 30)
    args = Arguments.from_dict({"x": {"client_num_in_total": 4, "iteration_number": 30, "mode": "DOL",
                                      "learning_rate": 0.05, "b_symmetric": True,
                                      "topology_neighbors_num_undirected": 2, "epoch": 1}})
    api = DecentralizedFLAPI(args, torch.device("cpu"), (X, Y), LogisticRegression(18, 2))
    reg = api.train()["regret"]
    assert reg[-1] < reg[0]
