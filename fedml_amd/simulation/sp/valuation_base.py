"""Shared machinery of the Shapley-valued FedAvg variants (S-FedAvg, HS-FedAvg):
dataset-tuple parsing, class-balanced loss weights, coalition valuation per round."""
import copy
import logging
import time
from collections import Counter

import numpy as np
import torch

from ...core.valuation import BatchedModelEvaluator, CoalitionValuer
from ...trainers import create_model_trainer
from ..common import save_results
from .fedavg.fedavg_api import FedAvgAPI


def calc_class_weight(train_data, class_num):
    """Balanced CE weights n / (n_unique · count_c), 0 for classes absent on the client
    (reference `s_fedavg/fedavg_api.py:112-136`, without the hard-coded dataset→class table)."""
    ys = torch.cat([y.reshape(-1) for _, y in train_data]).tolist() if len(train_data) else []
    cnt = Counter(ys)
    n, u = len(ys), len(cnt)
    return torch.tensor([n / (u * cnt[c]) if cnt.get(c) else 0.0 for c in range(int(class_num))],
                        dtype=torch.float32)


def s_fedavg_sampling(round_idx, client_num_in_total, client_num_per_round, phi=None, sampling_filter=None):
    """S-FedAvg client sampling (reference `s_fedavg/fedavg_api.py:435-477`): ``p ∝ exp(φ)`` when
    ``sampling_filter == "exp"``, else uniform, drawn from numpy's global generator (seeded by ``fedml.init``);
    every client when all of them take part."""
    if client_num_in_total == client_num_per_round:
        return list(range(client_num_in_total))
    n = min(client_num_per_round, client_num_in_total)
    if sampling_filter == "exp" and phi is not None:
        P = np.exp(np.asarray(phi, dtype=np.float64))
    else:
        P = np.ones(client_num_in_total)
    P = P / (P.sum() + 1e-13)
    return np.random.choice(range(client_num_in_total), size=n, replace=False, p=P).tolist()


def hs_fedavg_sampling(round_idx, client_num_in_total, client_num_per_round, phi=None):
    """HS-FedAvg client selection (reference `hs_fedavg/fedavg_api.py:284-302`): the top-K clients by φ, ties
    broken randomly (the reference picks a random sort algorithm); uniform ``np.random.seed(round)`` sampling
    while every φ is equal."""
    if client_num_in_total == client_num_per_round:
        return list(range(client_num_in_total))
    n = min(client_num_per_round, client_num_in_total)
    if phi is None or len(set(phi)) == 1:
        np.random.seed(round_idx)
        return np.random.choice(range(client_num_in_total), n, replace=False).tolist()
    rng = np.random.RandomState(round_idx)
    keys = np.lexsort((rng.random_sample(len(phi)), np.asarray(phi)))
    return keys[-n:].tolist()


def valuation_config(args, dataset=None):
    """(valid, alpha, beta, filter, approaching, score, target) from the reference's 15-tuple dataset or the
    config (`s_fedavg/fedavg_api.py:29-45`)."""
    ds = list(dataset) if dataset is not None else []
    if len(ds) >= 15:
        return tuple(ds[8:15])
    return (getattr(args, "valid_data_in_aggregator", None),
            float(getattr(args, "sv_alpha", getattr(args, "alpha", 0.5))),
            float(getattr(args, "sv_beta", getattr(args, "beta", 0.5))),
            getattr(args, "sampling_filter", "exp"),
            bool(getattr(args, "sv_approaching", False)),
            getattr(args, "score_method", "acc"),
            ds[8] if len(ds) == 9 else getattr(args, "target_label", None))


def validation_subset(test_global, n, seed, batch_size):
    """The server-side validation set: a seeded random subset of the global test set, as (x, y) batches."""
    xs, ys = [], []
    for x, y in test_global:
        xs.append(x)
        ys.append(y)
    if not xs:
        return []
    x, y = torch.cat(xs), torch.cat(ys)
    g = torch.Generator().manual_seed(int(seed))
    idx = torch.randperm(len(x), generator=g)[:n]
    bs = int(batch_size)
    return [(x[idx[i:i + bs]], y[idx[i:i + bs]]) for i in range(0, len(idx), bs)]


class ValuedFedAvgBase(FedAvgAPI):
    def __init__(self, args, device, dataset, model, model_trainer=None):
        ds = list(dataset)
        valid, alpha, beta, filt, approaching, score, target = valuation_config(args, ds)
        trainer = model_trainer or create_model_trainer(model, args)
        if hasattr(trainer, "clip_grad_norm"):
            trainer.clip_grad_norm = 1.0
        super().__init__(args, device, ds[:8] + [target], model, trainer)
        if valid is None:
            valid = self._validation_subset(int(getattr(args, "valid_samples", 10000)))
        self.global_valid_data = valid
        self.alpha, self.beta = float(alpha), float(beta)
        self.sampling_filter = filt
        self.sv_approaching = bool(approaching)
        self.score = str(score)
        self.seed = int(getattr(args, "random_seed", 0) or 0)
        self.evaluator = BatchedModelEvaluator(self.model_trainer.model, device,
                                               max_models=int(getattr(args, "sv_batch_models", 128)))

    def _validation_subset(self, n):
        """Random subset of the global test set as the server-side validation set."""
        return validation_subset(self.test_global, n, int(getattr(self.args, "random_seed", 0) or 0),
                                 int(self.args.batch_size))

    def _train_clients(self, client_indexes, w_global, **kw):
        w_locals = []
        for idx, client in enumerate(self.client_list):
            cid = int(client_indexes[idx])
            client.update_local_dataset(cid, self.train_data_local_dict[cid], self.test_data_local_dict[cid],
                                        self.train_data_local_num_dict[cid])
            self.model_trainer.class_weight = calc_class_weight(self.train_data_local_dict[cid], self.class_num)
            w_locals.append((client.get_sample_number(), self._client_train(client, copy.deepcopy(w_global), **kw)))
        self.model_trainer.class_weight = None
        return w_locals

    def _client_train(self, client, w, **kw):
        return client.train(w)

    def _valuer(self, w_locals):
        flats = torch.stack([self.evaluator.flatten(w) for _, w in w_locals])
        return CoalitionValuer(self.evaluator, flats, [n for n, _ in w_locals], self.global_valid_data,
                               self.score, self.target_label if isinstance(self.target_label, int) else None)

    def _finish_round(self, round_idx, w_locals, res_dict):
        w_global = self._aggregate(w_locals)
        self.model_trainer.set_model_params(w_global)
        freq = int(getattr(self.args, "frequency_of_the_test", 1) or 1)
        if round_idx == int(self.args.comm_round) - 1 or round_idx % freq == 0:
            res_dict[round_idx] = self._local_test_on_all_clients(round_idx)
        res_dict.setdefault(round_idx, {})
        acc, recall = self._validate_global_model(self.model_trainer.model, self.test_global, self.device)
        res_dict[round_idx]["Global/Acc"], res_dict[round_idx]["Global/Recall"] = acc, recall
        return w_global

    def _dump(self, **dicts):
        out = getattr(self.args, "results_path", None)
        if out:
            save_results(dicts, out)
        self.results = dicts
