"""UCI streaming data for decentralized online learning (reference: ``data/UCI/data_loader_for_susy_and_ro.py``).

SUSY (``label,f1..f18`` rows) and Room Occupancy (``id,date,f1..f5,label`` rows) CSV files become one
sample stream per client:
  * the first ``beta`` fraction of the samples is clustered with k-means into one cluster per client and
    each cluster goes to its client (the "adversarial", non-IID part of the stream);
  * the remaining samples fill the clients in order up to ``sample_num_in_total / n_clients`` each
    (the "stochastic" part); longer adversarial streams are cut to that length and their surplus joins
    the stochastic pool first, as in the reference.
Returns ``{client: (X [T_c, d] float32, Y [T_c] int64)}`` and ``stack_streams`` turns it into the
``[N, T, d]`` / ``[N, T]`` tensors ``DecentralizedFLAPI`` consumes (truncated to the shortest stream)."""
import csv
from typing import Dict, List, Tuple

import numpy as np
import torch


def read_uci_csv(path: str, data_name: str, limit: int):
    X, Y = [], []
    with open(path) as f:
        for i, row in enumerate(csv.reader(f, delimiter=",")):
            if i >= limit:
                break
            if data_name == "SUSY":
                X.append(np.asarray(row[1:], dtype=np.float32))
                Y.append(int(row[0].split(".")[0]))
            elif data_name == "RO":
                X.append(np.asarray(row[2:-1], dtype=np.float32))
                Y.append(int(row[-1].split(".")[0]))
            else:
                raise ValueError(f"data_name {data_name!r}: SUSY | RO")
    return np.stack(X), np.asarray(Y, dtype=np.int64)


def load_streams(path: str, data_name: str, client_list: List[int], sample_num_in_total: int, beta: float,
                 seed: int = 0) -> Dict[int, Tuple[torch.Tensor, torch.Tensor]]:
    X, Y = read_uci_csv(path, data_name, sample_num_in_total)
    n_cl = len(client_list)
    per = sample_num_in_total // n_cl
    streams = {c: [] for c in client_list}
    n_adv = int(sample_num_in_total * beta) if beta > 0 else 0
    n_adv = min(n_adv, len(X))
    if n_adv:
        from sklearn.cluster import KMeans
        lab = KMeans(n_clusters=n_cl, n_init=10, random_state=seed).fit(X[:n_adv]).labels_
        for i, k in enumerate(lab):
            streams[client_list[int(k)]].append(i)
    pool = list(range(n_adv, len(X)))
    surplus = []
    for c in client_list:   # adversarial streams longer than the per-client length give their tail back
        if len(streams[c]) > per:
            surplus += streams[c][per:]
            streams[c] = streams[c][:per]
    pool = surplus + pool
    j = 0
    for c in client_list:
        while len(streams[c]) < per and j < len(pool):
            streams[c].append(pool[j])
            j += 1
    return {c: (torch.from_numpy(X[idx]) if idx else torch.zeros(0, X.shape[1]),
                torch.from_numpy(Y[idx]) if idx else torch.zeros(0, dtype=torch.int64))
            for c, idx in streams.items()}


def stack_streams(streams) -> Tuple[torch.Tensor, torch.Tensor]:
    T = min(len(v[0]) for v in streams.values())
    keys = sorted(streams)
    return torch.stack([streams[k][0][:T] for k in keys]), torch.stack([streams[k][1][:T] for k in keys])
