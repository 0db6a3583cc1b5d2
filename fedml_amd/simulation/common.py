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


def class_rates(tp, actual, predicted):
    """Per-class (recall, precision) dicts of one evaluation, the fork's formula
    (``my_model_trainer_classification.py:148-153``): over the classes present in the labels,
    (tp + 1e-13) / (den + 1e-13), set to 0 below 1e-13 — a class that was never predicted gets precision 1.
    Deviation: the fork counts a class's predictions only in batches whose labels contain it (its
    denominator depends on the batch split); here they are counted over the whole evaluation."""
    tp, actual, predicted = (np.asarray(v, dtype=np.float64).reshape(-1) for v in (tp, actual, predicted))
    rec, prec = {}, {}
    for k in np.nonzero(actual > 0)[0].tolist():
        r = (tp[k] + 1e-13) / (actual[k] + 1e-13)
        p = (tp[k] + 1e-13) / (predicted[k] + 1e-13)
        rec[int(k)] = 0.0 if r < 1e-13 else float(r)
        prec[int(k)] = 0.0 if p < 1e-13 else float(p)
    return rec, prec


def fork_local_test_stats(train_m, test_m):
    """The per-round dict of ``_local_test_on_all_clients`` (fork ``fedavg_api.py:238-326``) from per-client
    metric dicts (``test_correct``, ``test_total``, ``test_loss`` and, for test data, ``test_recall`` /
    ``test_precision``): the federation-wide scalars (also under the reference's wandb names
    ``Train/Acc`` ... ``Test/Loss``, which the fork logs as scalars) plus the per-client lists. Naming: the fork
    returns its per-client accuracy lists under ``Test/Acc`` / ``Train/Acc``; here those keys keep the scalar
    (wandb) meaning and the lists are ``Test/AccPerClient`` / ``Train/AccPerClient``."""
    tr_acc, tr_loss = summarize_metrics(train_m)
    te_acc, te_loss = summarize_metrics(test_m)

    def per_client(ms):
        return [m.get("test_correct", 0) / m["test_total"] if m.get("test_total") else 0.0 for m in ms]
    return {"Train/Acc": tr_acc, "Train/Loss": tr_loss, "Test/Acc": te_acc, "Test/Loss": te_loss,
            "Authority/Train/Acc": tr_acc, "Authority/Test/Acc": te_acc,
            "Train/AccPerClient": per_client(train_m), "Test/AccPerClient": per_client(test_m),
            "Test/Recall": [m.get("test_recall", {}) for m in test_m],
            "Test/Precision": [m.get("test_precision", {}) for m in test_m]}


def scalar_metrics(rec: dict) -> dict:
    """The scalar entries of a metrics record (what goes to the log line and the metrics sink)."""
    return {k: v for k, v in rec.items() if isinstance(v, (int, float)) or v is None}


def log_metrics(metrics: dict, round_idx: int):
    from ..core.mlops import MLOpsMetrics
    metrics = scalar_metrics(metrics)
    logging.info("round %d: %s", round_idx, {k: (round(v, 5) if isinstance(v, float) else v) for k, v in metrics.items()})
    MLOpsMetrics.get_instance().log(dict(metrics, round=round_idx), step=round_idx)
