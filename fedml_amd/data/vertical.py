"""Vertically partitioned tabular data (stand-in for lending_club_loan / NUS-WIDE / UCI, which
cannot be downloaded here). Features are split column-wise across parties; party 0 (guest)
holds the labels. Labels follow a logistic model over ALL parties' features, so no single
party can fit them alone — the property a VFL test needs."""
import numpy as np
import torch


def synthetic_vertical(n_train=2000, n_test=500, party_dims=(10, 10, 10), seed=0, noise=0.1):
    rng = np.random.default_rng(seed)
    d = int(sum(party_dims))
    w = rng.normal(size=d).astype(np.float32)
    X = rng.normal(size=(n_train + n_test, d)).astype(np.float32)
    logits = X @ w / np.sqrt(d) * 3 + rng.normal(scale=noise, size=n_train + n_test)
    y = (logits > 0).astype(np.float32)
    parts, o = [], 0
    for k in party_dims:
        parts.append(torch.from_numpy(X[:, o:o + k].copy()))
        o += k
    ytr, yte = torch.from_numpy(y[:n_train]), torch.from_numpy(y[n_train:])
    train = [p[:n_train] for p in parts]
    test = [p[n_train:] for p in parts]
    return train, ytr, test, yte
