"""S-FedAvg and HS-FedAvg on the RCCL virtual-client engine (the fork's defining algorithms).

Reference (sequential, one client after another on one shared model, a ``deepcopy`` of the global state per client):
`single_process/s_fedavg/fedavg_api.py:148-358` (train loop), `:435-477` (p ∝ exp(φ) sampling),
`s_fedavg/my_model_trainer_classification.py:27,57` (class-balanced CE, clip 1.0),
`hs_fedavg/fedavg_api.py:135,171-175,284-302` (amplitude sharing, top-K by φ), `hs_fedavg/hs_fft.py:8-84`.

Here a round is the FedAvg round of ``RCCLSimulator`` — every sampled client of a GPU trains at once in the client-
batched engine (native HIP ResNet step / batched interpreter / sequential executor) — with the valued variants'
pieces slotted in:

* sampling: S-FedAvg draws ``p ∝ exp(φ)`` (``sampling_filter: exp``) from numpy's global generator, HS-FedAvg takes
  the top-K by φ (same functions as the SP simulator, ``sp/valuation_base.py``) — rank 0's draw is broadcast;
* local training: per-client class-balanced CE as per-row loss scales (``engine.class_weight``, one [C, classes]
  table gathered per round from a device-side per-client label histogram) and the per-client gradient clip 1.0
  inside the (captured) optimizer step; HS-FedAvg normalises every client's batches toward its running Fourier
  amplitude on the device (``ops.spectral`` K12 kernels, ``engine.input_hook``), and the clients' amplitudes are
  averaged with one all-reduce;
* valuation: the K trained models are all-gathered ([K, P], one collective), every coalition average is one
  ``[S, K] × [K, P]`` MFMA product (``ops.subset_aggregate``), and the coalition evaluations are SHARDED over the
  ranks (``CoalitionValuer(shard=True)``: coalition i on rank i mod W, scores all-gathered); exact (reference
  estimator) or Monte-Carlo permutation Shapley values, then ``φ ← α·φ + β·sv`` (S: sv replaced, HS: accumulated).
"""
import logging
import time

import numpy as np
import torch

from ...constants import FedML_FEDERATED_OPTIMIZER_HS_FEDAVG
from ...core.schedule import pack_clients_to_gpus
from ...core.valuation import BatchedModelEvaluator, CoalitionValuer
from ...parallel import comm
from ..sp.valuation_base import hs_fedavg_sampling, s_fedavg_sampling, validation_subset, valuation_config
from .simulator import RCCLSimulator


def class_weight_table(store, num_classes: int) -> torch.Tensor:
    """[K_total, classes] balanced CE weights n / (n_unique · count_c) per client (0 for absent classes), from the
    device store's labels in one histogram — the reference's `s_fedavg/fedavg_api.py:112-136` per client."""
    K = store.num_clients
    counts = store.counts
    cid = torch.repeat_interleave(torch.arange(K, device=store.device), counts)
    lab = store.y_all.reshape(len(store.y_all), -1)[:, 0].long()
    hist = torch.bincount(cid * num_classes + lab, minlength=K * num_classes).view(K, num_classes).double()
    n = counts.double().view(K, 1)
    u = (hist > 0).sum(1, keepdim=True).double()
    w = torch.where(hist > 0, n / (u * hist.clamp_min(1)), torch.zeros_like(hist))
    return w.float()


class ValuedRCCLSimulator(RCCLSimulator):
    def __init__(self, args, device, dataset, model, store=None, model_trainer=None, valid_data=None):
        self.variant = str(args.federated_optimizer)
        valid, alpha, beta, filt, approaching, score, target = valuation_config(args, dataset)
        if model_trainer is not None and not getattr(model_trainer, "functional", False):
            raise ValueError(f"{self.variant} on the RCCL simulator trains through the engine (functional trainers)")
        args.clip_grad_norm = 1.0          # reference s_fedavg/my_model_trainer_classification.py:57
        super().__init__(args, device, dataset, model, store=store, model_trainer=model_trainer)
        self.hs = self.variant == FedML_FEDERATED_OPTIMIZER_HS_FEDAVG
        self.alpha, self.beta = float(alpha), float(beta)
        self.sampling_filter = filt
        self.sv_approaching = bool(approaching) and not self.hs
        self.score = str(score)
        self.target = target if isinstance(target, int) else None
        seed = int(getattr(args, "random_seed", 0) or 0)
        if valid_data is not None:
            valid = valid_data
        if valid is None:
            if dataset is None:
                raise ValueError(f"{self.variant}: no validation data (pass valid_data or a dataset)")
            valid = validation_subset(dataset[3], int(getattr(args, "valid_samples", 10000)), seed,
                                      int(args.batch_size))
        self.valid = [(x.to(self.device), y.to(self.device)) for x, y in valid]
        self.evaluator = BatchedModelEvaluator(self.model, self.device,
                                               max_models=int(getattr(args, "sv_batch_models", 128)),
                                               compute_dtype=self.compute_dtype)
        K = self.K_total
        self.phi = [1.0 / K] * K
        self.sv = [(1 - self.alpha) / (K * self.beta)] * K
        ncls = int(dataset[7]) if dataset is not None else 0
        ncls = max(ncls, int(self.store.y_all.max()) + 1)
        self.cw_table = class_weight_table(self.store, ncls)
        self.mc_rng = np.random.RandomState((seed * 7919 + 17) & 0xFFFFFFFF)
        self.results = {"phi": {}, "sv": {}, "client": {}, "time": {}, "sampled": {}}
        self.amp_summary = None
        self.amp_momentum = float(getattr(args, "amp_momentum", 0.1))
        self.amp_band = float(getattr(args, "amp_band", 0.0))
        self._assigned = None

    # ------------------------------------------------------------------------------------------
    def assignment(self, round_idx: int):
        if self._assigned is not None and self._assigned[0] == round_idx:
            return self._assigned[1], self._assigned[2]
        if self.hs:
            ids = hs_fedavg_sampling(round_idx, self.K_total, self.K, self.phi)
        else:
            ids = s_fedavg_sampling(round_idx, self.K_total, self.K, self.phi, self.sampling_filter)
        ids = [int(i) for i in ids]
        if comm.is_dist():
            # rank 0's draw is THE sample: a rank whose numpy state drifted (extra rank-local draws, another resume
            # path) would otherwise pack different clients and desynchronise every later collective
            t = torch.tensor(ids, dtype=torch.int64, device=self.device)
            comm.broadcast_flat(t, 0)
            ids = [int(i) for i in t.tolist()]
        packs = pack_clients_to_gpus([self.sample_counts[i] for i in ids], self.world)
        self.packs = [[ids[j] for j in pk] for pk in packs]
        mine = self.packs[self.rank]
        self.round_owner = {c: r for r, pk in enumerate(self.packs) for c in pk}
        self._assigned = (round_idx, ids, mine)
        return ids, mine

    def _amp_hook(self, amps, touched):
        def hook(x, b_c):
            if x.dim() != 5:
                return x
            from ...ops.spectral import amplitude_normalize
            for c, b in enumerate(b_c):
                if b > 0:
                    out, amps[c] = amplitude_normalize(x[c, :b], amps[c], self.amp_momentum, False, self.amp_band)
                    x[c, :b] = out
                    touched[c] = True
            return x
        return hook

    def run_round(self, round_idx: int):
        ids, mine = self.assignment(round_idx)
        C = self.C
        cw = torch.zeros(C, self.cw_table.shape[1], dtype=torch.float32, device=self.device)
        if mine:
            cw[:len(mine)] = self.cw_table[torch.as_tensor(mine, device=self.device)]
        self.engine.class_weight = cw
        amps = touched = None
        if self.hs:
            H, W = self.store.x_all.shape[-2], self.store.x_all.shape[-1]
            ch = self.store.x_all.shape[1]
            init = self.amp_summary if self.amp_summary is not None else torch.zeros(ch, H, W, device=self.device)
            amps = [init.clone() for _ in range(C)]
            touched = [False] * C
            self.engine.input_hook = self._amp_hook(amps, touched)
        try:
            super().run_round(round_idx)
        finally:
            self.engine.input_hook = None
        if self.hs:
            self._share_amplitudes(amps, touched, len(mine))
        t0 = time.perf_counter()
        stack = self._gather_models(ids)
        n = [self.sample_counts[c] for c in ids]
        valuer = CoalitionValuer(self.evaluator, stack, n, self.valid, self.score, self.target, shard=True)
        if self.sv_approaching:
            round_sv = valuer.monte_carlo_sv(self.mc_rng)
        else:
            round_sv = valuer.exact_reference_sv()
        valuer.ensure([1 << i for i in range(len(ids))])
        client = {}
        for i, cid in enumerate(ids):
            m = valuer.metrics[1 << i]
            client[cid] = m["correct"] / max(1.0, m["total"])
            self.sv[cid] = self.sv[cid] + round_sv[i] if self.hs else round_sv[i]
            self.phi[cid] = self.alpha * self.phi[cid] + self.beta * self.sv[cid]
        dt = time.perf_counter() - t0
        r = self.results
        r["client"][round_idx], r["time"][round_idx], r["sampled"][round_idx] = client, dt, list(ids)
        r["phi"][round_idx], r["sv"][round_idx] = list(self.phi), list(self.sv)
        if self.rank == 0:
            logging.info("[%s/RCCL] round %d: valuation of %d clients %.3fs (%d coalition models)", self.variant,
                         round_idx, len(ids), dt, valuer.evaluations)

    def _gather_models(self, ids):
        """[K, P] trained client models in sampled order (coalition bit i ↔ ids[i]): one all-gather of every
        rank's [C, P] client stack."""
        P = self.layout.size
        if comm.is_dist():
            parts = comm.all_gather_flat(self.engine.params.reshape(-1))
            rows = {c: parts[r].view(self.C, P)[j] for r, pk in enumerate(self.packs) for j, c in enumerate(pk)}
        else:
            rows = {c: self.engine.params[j] for j, c in enumerate(self.packs[0])}
        return torch.stack([rows[c] for c in ids])

    def _share_amplitudes(self, amps, touched, n_mine):
        """amp_summary = mean of the sampled clients' running amplitudes (reference `hs_fedavg/fedavg_api.py:
        171-175`); a client that never trained keeps no amplitude unless one was handed to it."""
        ch, H, W = amps[0].shape
        acc = torch.zeros(ch * H * W + 1, dtype=torch.float32, device=self.device)
        for c in range(n_mine):
            if touched[c] or self.amp_summary is not None:
                acc[:-1] += amps[c].reshape(-1)
                acc[-1] += 1
        comm.all_reduce_flat(acc)
        cnt = float(acc[-1])
        if cnt > 0:
            self.amp_summary = (acc[:-1] / cnt).view(ch, H, W)
