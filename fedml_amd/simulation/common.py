"""Helpers shared by every simulator: reference-exact client sampling, results sinks,
metric aggregation over clients."""
import json
import logging
import os

import numpy as np


def client_sampling(round_idx, client_num_in_total, client_num_per_round):
    """`np.random.seed(round_idx); np.random.choice(range(N), K, replace=False)`; all clients if K == N
    (reference: `single_process/fedavg/fedavg_api.py:179-193`)."""
    if client_num_in_total == client_num_per_round:
        return list(range(client_num_in_total))
    num_clients = min(client_num_per_round, client_num_in_total)
    np.random.seed(round_idx)
    return [int(i) for i in np.random.choice(range(client_num_in_total), num_clients, replace=False)]


def data_silo_selection(round_idx, client_num_in_total, client_num_per_round):
    """Cross-silo variant (reference: `cross_silo/horizontal/fedml_aggregator.py:103-140`): each silo
    picks a data index from the dataset's clients (with replacement when silos > data clients)."""
    if client_num_in_total == client_num_per_round:
        return list(range(client_num_per_round))
    np.random.seed(round_idx)
    return [int(i) for i in np.random.choice(range(client_num_in_total), client_num_per_round,
                                             replace=client_num_per_round > client_num_in_total)]


def save_results(res, path):
    """Results as JSON (the reference joblib-pickles `.tmp_res*.pkl`; JSON is loadable without pickle)."""
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)

    def conv(o):
        if isinstance(o, (np.integer,)):
            return int(o)
        if isinstance(o, (np.floating,)):
            return float(o)
        if hasattr(o, "tolist"):
            return o.tolist()
        return str(o)

    with open(path, "w") as f:
        json.dump(res, f, default=conv, indent=1)
    return path


def summarize_metrics(per_client):
    """Sum test_correct/test_total/test_loss over clients → (acc, loss)."""
    correct = sum(m.get("test_correct", 0) for m in per_client)
    total = sum(m.get("test_total", 0) for m in per_client)
    loss = sum(m.get("test_loss", 0.0) for m in per_client)
    return (correct / total if total else 0.0), (loss / total if total else 0.0)


def log_metrics(metrics: dict, round_idx: int):
    from ..core.mlops import MLOpsMetrics
    logging.info("round %d: %s", round_idx, {k: (round(v, 5) if isinstance(v, float) else v) for k, v in metrics.items()})
    MLOpsMetrics.get_instance().log(dict(metrics, round=round_idx), step=round_idx)
