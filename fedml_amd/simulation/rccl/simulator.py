"""Parrot-RCCL: the MI355X-native FL simulator (reference NCCL simulator is a stub,
`simulation/simulator.py:100-108`; intent: "AllReduce-based FL with resource scheduling",
`simulation/nccl/README.md`).

One process per GPU. Per round:
  1. every rank derives the same client sample (reference RNG: ``np.random.seed(round)``) and the
     same client→GPU packing (native branch-and-bound scheduler, ``core.schedule``);
  2. each rank expands the global flat model into its [C, P] client stack and trains all its
     virtual clients at once (``ClientBatchEngine``);
  3. each rank reduces its clients to Σ n_c·w_c ‖ Σ n_c on-GPU (FedAvg kernel) and ONE RCCL
     all-reduce over xGMI produces the next global model on every rank (no server process,
     no per-client messages, no pickling);
  4. optional server optimizer (FedOpt: fused HIP kernel), robust aggregation, evaluation,
     checkpointing.
"""
import copy
import logging
from collections.abc import Mapping
import math
import os
import time
from typing import Dict, List, Optional

import numpy as np
import torch

from ... import ops
from ...core.arena import ParamLayout
from ...core.fault import FaultInjector
from ...core.mlops import MLOpsMetrics
from ...core.schedule import pack_clients_to_gpus
from ...core.tracing import tracer
from ...parallel import comm
from ..common import client_sampling
from .client_store import DeviceClientStore
from .engine import ClientBatchEngine
from .residuals import ShardedResiduals


class _LazyState(Mapping):
    """Read-only state-dict view of a flat global-model snapshot; unflattened on the host on first access."""

    def __init__(self, layout, flat):
        self._layout, self._flat, self._sd = layout, flat, None

    def _get(self):
        if self._sd is None:
            self._sd = self._layout.unflatten(self._flat.cpu())
            self._flat = None
        return self._sd

    def __getitem__(self, k):
        return self._get()[k]

    def __iter__(self):
        return iter(self._get())

    def __len__(self):
        return len(self._get())


def _dtype(name):
    """compute_dtype config value → engine compute dtype (None = fp32, the reference's precision)."""
    table = {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp16": torch.float16, "float16": torch.float16,
             "fp32": None, "float32": None, None: None}
    if name not in table:
        raise ValueError(f"compute_dtype {name!r}: expected one of fp32 | bf16 | fp16")
    return table[name]


def fednova_normalizer(tau: int, lr: float, momentum: float = 0.0, mu: float = 0.0):
    """(a_i, τ_eff_i / p_i) of a client after ``tau`` local SGD steps — the counters of the FedNova local
    optimizer (``trainers/fednova.py``, reference ``single_process/fednova/fednova.py:110-140``): with
    momentum ρ each step adds the geometric counter 1 + ρ + … ; a proximal term μ damps the running sum by
    (1 − lr·μ) per step; plain SGD counts steps. τ_eff_i is τ·p_i under a proximal term, else a_i·p_i."""
    vec, counter, etamu = 0.0, 0.0, lr * mu
    for _ in range(int(tau)):
        if momentum:
            counter = counter * momentum + 1.0
            vec += counter
        if etamu:
            vec = vec * (1.0 - etamu) + 1.0
        if not momentum and not etamu:
            vec += 1.0
    return vec, (float(tau) if mu else vec)


_PEER_FAILURE_MARKERS = ("connection closed", "connection reset", "connection refused", "broken pipe", "peer",
                         "gloo", "nccl", "rccl", "timed out", "timeout", "socket", "communicator")


def _is_peer_failure(e: BaseException) -> bool:
    """A collective that failed because another rank died or became unreachable (what elastic re-init
    can repair), as opposed to a local error."""
    if isinstance(e, torch.distributed.DistBackendError):
        return True
    msg = str(e).lower()
    return any(m in msg for m in _PEER_FAILURE_MARKERS)


class RCCLSimulator:
    def __init__(self, args, device, dataset, model, store: Optional[DeviceClientStore] = None, model_trainer=None):
        """``model_trainer`` (reference ``fedml.run_simulation(..., model_trainer)``): a functional trainer
        (``FunctionalTrainerMixin``: standard supervised SGD/Adam with a named loss) configures the
        client-batched engine (loss_name, clip_grad_norm); any other ``ClientTrainer`` runs its own
        ``train()`` per client (compatibility path) and only aggregation stays on the GPU."""
        self.args = args
        self.user_trainer = None
        if model_trainer is not None:
            if getattr(model_trainer, "functional", False):
                args.loss_name = getattr(model_trainer, "loss_name", "ce")
                if getattr(model_trainer, "clip_grad_norm", None) is not None:
                    args.clip_grad_norm = model_trainer.clip_grad_norm
            else:
                self.user_trainer = model_trainer
        self.device = torch.device(device)
        from ...utils import determinism
        if determinism.enabled(args):
            determinism.enable(args)     # before the process group: the RCCL env must precede the communicator
        self.rank, self.world = comm.init_process_group(device=self.device if self.device.type == "cuda" else None,
                                                        args=args)
        self.model = model.to(self.device)
        self.dataset = dataset
        self.K_total = int(args.client_num_in_total)
        self.K = int(args.client_num_per_round)
        self.C = math.ceil(self.K / self.world)
        self.compute_dtype = _dtype(getattr(args, "compute_dtype", None)) if self.device.type == "cuda" else None
        if dataset is not None:
            train_local = dataset[5]
            self.sample_counts = [int(dataset[4][c]) for c in range(self.K_total)]
        else:
            train_local = None
            self.sample_counts = None
        with tracer().span("store.build"):
            self.store = store if store is not None else DeviceClientStore.from_client_data(train_local, self.device)
        if self.sample_counts is None:
            self.sample_counts = self.store.counts_host
        self.engine = ClientBatchEngine(self.model, self.C, self.device, args, self.compute_dtype)
        self.layout: ParamLayout = self.engine.layout
        self.global_flat = self.layout.flatten(self.model.state_dict(), device=self.device)
        comm.broadcast_flat(self.global_flat, 0)
        self.partial = torch.empty(self.layout.size + 1, dtype=torch.float32, device=self.device)
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(getattr(args, "random_seed", 0)) * 7777 + self.rank)
        self.server_opt = None
        if str(args.federated_optimizer) == "FedOpt":
            self.server_opt = _ServerOptState(args, self.layout.size, self.device)
        # FedNova: normalised averaging (coefficients from each client's local step count) + optional server
        # momentum gmf, applied by the fused K11 kernel on the all-reduced weighted sum
        self.fednova = str(args.federated_optimizer) == "FedNova"
        self.nova_gmf = float(getattr(args, "gmf", 0.0) or 0.0) if self.fednova else 0.0
        self.nova_buf = torch.zeros(self.layout.size, dtype=torch.float32, device=self.device) \
            if self.nova_gmf else None
        self.nova_first = True
        # the reference re-creates its global momentum buffer every round (fednova_trainer.py:80), so gmf
        # reduces to w −= cum_grad; `fednova_gmf_persist: true` keeps the buffer across rounds instead
        self.nova_persist = bool(getattr(args, "fednova_gmf_persist", False))
        self.round_times: List[float] = []
        # aggregation bucket (elements) for the pipelined weighted-sum + all-reduce of large models
        self.bucket_elems = max(256, int(float(getattr(args, "allreduce_bucket_mb", 32) or 32) * (1 << 20) / 4))
        # update compression (north-star config: FedOpt + int8/fp8/top-k with error feedback)
        self.compression = str(getattr(args, "compression", "") or "").lower() or None
        self.compress_ratio = float(getattr(args, "compression_ratio", 0.01) or 0.01)
        # error-feedback residuals: one row per client, on the rank that trains it (residuals.py)
        self.residual = ShardedResiduals(self.layout.size, self.device, self.rank, self.world) \
            if self.compression else None
        self.upload_bytes: List[int] = []
        self.faults = FaultInjector(args)
        self.dropped_clients: List[int] = []
        self.history: Dict[int, dict] = {}
        self.round_idx = 0
        # elastic: survive a dead peer by rebuilding the communicator from the survivors (parallel/elastic.py)
        self.elastic = bool(getattr(args, "elastic", False)) and comm.is_dist()
        if self.elastic:
            if self.compression:
                raise ValueError("elastic re-init does not support compressed updates (residual rows of a dead "
                                 "rank are lost)")
            from ...parallel import elastic
            elastic.setup(self.rank, self.world, str(torch.distributed.get_backend()),
                          int(getattr(args, "elastic_timeout_s", 60) or 60))
        self.world_changes: List[tuple] = []

    # ---------------------------------------------------------------------------------------------
    def assignment(self, round_idx: int):
        ids = client_sampling(round_idx, self.K_total, self.K)
        counts = [self.sample_counts[i] for i in ids]
        packs = pack_clients_to_gpus(counts, self.world)
        mine = [ids[j] for j in packs[self.rank]]
        self.round_owner = {int(ids[j]): r for r, pk in enumerate(packs) for j in pk}   # client → rank
        return ids, mine

    def run_round(self, round_idx: int):
        tr = tracer()
        args = self.args
        with tr.span("round.assign"):
            ids, mine = self.assignment(round_idx)
            slots = torch.full((self.C,), 0, dtype=torch.int64)
            valid = torch.zeros(self.C, dtype=torch.bool)
            for i, cid in enumerate(mine):
                slots[i] = cid
                valid[i] = True
            slots = slots.to(self.device)
            valid = valid.to(self.device)
        if self.fednova and (self.compression or self.server_opt is not None or self.user_trainer is not None):
            raise ValueError("FedNova on the RCCL simulator: compressed updates, a server optimizer or a user "
                             "ClientTrainer are not supported")
        if self.residual is not None:
            with tr.span("round.residual_migrate"):
                self.residual.migrate(self.round_owner)
        with tr.gpu_span("round.broadcast_local", self.device):
            self.engine.load_global(self.global_flat)
        with tr.gpu_span("round.local_train", self.device):
            # data order / augmentation keyed by (seed, round, client): identical for any world size and
            # exactly reproducible on resume from the round index alone
            rng_key = (int(getattr(args, "random_seed", 0)) * 1000003 + int(round_idx) * 7919) & 0x7FFFFFFF
            if self.user_trainer is not None:
                self._train_user_trainer(mine)
            else:
                self.engine.train(self.store, slots, int(args.epochs), int(args.batch_size),
                                  float(args.learning_rate), generator=self.gen,
                                  shuffle=bool(getattr(args, "shuffle", True)), valid_slots=valid, rng_key=rng_key)
        with tr.gpu_span("round.aggregate", self.device):
            if self.fednova:
                w = self._fednova_coefficients(ids, mine)
                if not self.nova_persist:
                    self.nova_first = True
            else:
                w = torch.where(valid, self.store.counts[slots].to(torch.float32),
                                torch.zeros(self.C, device=self.device))
            if self.faults.active:
                # lost uploads (dropout / missed deadline, core.fault): survivors are re-weighted
                alive = self.faults.survivors(round_idx, mine)
                self.dropped_clients.append(int((~alive).sum()))
                keep = torch.zeros(self.C, dtype=torch.float32)
                keep[:len(mine)] = torch.from_numpy(alive.astype("float32"))
                w = w * keep.to(self.device)
            self._robust_preaggregate(w)
            if self.compression:
                ids = list(mine) + [-1] * (self.C - len(mine))     # -1: padding slot (no residual row)
                n_up = len(mine) if not self.faults.active else int(keep.sum())
                _, nb = self.engine.compressed_partial_sum(w, self.global_flat, ids, self.residual, self.compression,
                                                           self.compress_ratio, round_idx, out=self.partial,
                                                           n_upload=n_up)
                self.upload_bytes.append(nb)
                comm.all_reduce_flat(self.partial)
            elif self.engine.deterministic:
                self._det_partial_sum(w, normalize=not self.fednova)
            elif comm.is_dist() and self.layout.size > self.bucket_elems:
                # large models (DistilBERT / ViT: 67-86 M params): the weighted sum is produced bucket by
                # bucket and each bucket's all-reduce is enqueued at once — RCCL's stream reduces bucket k
                # over xGMI while this stream sums bucket k+1
                P = self.layout.size
                works = []
                for lo in range(0, P, self.bucket_elems):
                    hi = min(P, lo + self.bucket_elems)
                    ops.weighted_sum(self.engine.params[:, lo:hi], w, out=self.partial[lo:hi])
                    works += comm.all_reduce_flat(self.partial[lo:hi], async_op=True)
                self.partial[P:].copy_(w.sum().view(1))
                works += comm.all_reduce_flat(self.partial[P:], async_op=True)
                for wk in works:
                    wk.wait()
            else:
                self.engine.partial_sum(w, out=self.partial)
                comm.all_reduce_flat(self.partial)
            if self.fednova:
                # normalised update g − (S·g − Σ coef_i w_i) (+ server momentum), one fused pass
                P = self.layout.size
                ops.fednova_server_step(self.global_flat, self.partial[:P], self.partial[P:P + 1], self.nova_buf,
                                        self.nova_gmf, float(args.learning_rate), self.nova_first)
                self.nova_first = False
                self._post_aggregate()
                return
            total = self.partial[self.layout.size:self.layout.size + 1]
            avg = self.partial[:self.layout.size] / total.clamp_min(1e-12)
            if self.faults.active:   # every upload lost: the global model stays as it was
                avg = torch.where(total > 0, avg, self.global_flat)
            if self.server_opt is not None:
                self.server_opt.step(self.global_flat, avg)
            else:
                self.global_flat.copy_(avg)
            self._post_aggregate()

    def _det_partial_sum(self, w, normalize=True):
        """Deterministic mode: Σ_c w_c·params_c ‖ Σ_c w_c accumulated and all-reduced in fp64, rounded to fp32 once.
        The fp64 sums of different client groupings (1 rank × K clients vs R ranks × K/R) differ only at 2^-53, far
        below the final fp32 rounding, so the global model's bits do not depend on the world size (barring an fp64
        sum that lands within 2^-53 of an fp32 rounding tie).

        ``normalize``: the weighted MEAN is formed in fp64 too (one rounding to fp32 instead of rounding the sum and
        then dividing in fp32); ``partial`` then holds avg ‖ 1 (‖ 0 when every weight is zero), so the caller's
        ``partial[:P] / partial[P]`` is exact. FedNova (which needs the raw sums) passes False."""
        P = self.layout.size
        if getattr(self, "_partial64", None) is None:
            self._partial64 = torch.empty(P + 1, dtype=torch.float64, device=self.device)
        wd = w.to(torch.float64).view(-1, 1)
        step = max(1, (1 << 26) // max(1, self.C))         # bounds the fp64 temporary to 512 MB
        for lo in range(0, P, step):
            hi = min(P, lo + step)
            torch.sum(self.engine.params[:, lo:hi].to(torch.float64) * wd, 0, out=self._partial64[lo:hi])
        self._partial64[P:].copy_(wd.sum().view(1))
        comm.all_reduce_flat(self._partial64)
        if normalize:
            tot = self._partial64[P:]
            self.partial[:P].copy_(self._partial64[:P] / tot.clamp_min(1e-300))
            self.partial[P:].copy_((tot > 0).to(torch.float32))
        else:
            self.partial.copy_(self._partial64)

    def _fednova_coefficients(self, ids, mine):
        """FedNova weights of this rank's slots: coef_i = τ_eff·p_i / a_i with p_i = n_i / Σn over the round's
        sampled clients (all ranks — every rank computes the same host-side numbers, no communication) and
        a_i from the client's local step count τ_i = epochs·⌈n_i / batch⌉ (``fednova_normalizer``)."""
        a = self.args
        lr, bs, ep = float(a.learning_rate), int(a.batch_size), int(a.epochs)
        mom = self.engine.momentum if self.engine.optimizer == "sgd" else 0.0
        mu = self.engine.mu
        n_all = {int(c): int(self.sample_counts[int(c)]) for c in ids}
        total = float(sum(n_all.values())) or 1.0
        norm = {c: fednova_normalizer(ep * math.ceil(n / bs), lr, mom, mu) for c, n in n_all.items()}
        tau_eff = sum((n_all[c] / total) * norm[c][1] for c in n_all)
        coef = torch.zeros(self.C, dtype=torch.float32)
        for i, cid in enumerate(mine):
            a_i = norm[int(cid)][0]
            if a_i > 0:
                coef[i] = tau_eff * (n_all[int(cid)] / total) / a_i
        return coef.to(self.device)

    def _train_user_trainer(self, mine):
        """Compatibility path for a non-functional ``ClientTrainer`` (reference client.py:27-47 call
        order: set_id → set_model_params(global) → train(local data) → get_model_params): each of this
        rank's clients trains through the user's own loop; its weights land in the engine's slot so the
        weighted sum and the all-reduce run exactly as on the batched path."""
        if self.dataset is None:
            raise ValueError("a user ClientTrainer needs the dataset's per-client loaders (dataset[5])")
        tr = self.user_trainer
        glob = self.layout.unflatten(self.global_flat.detach().cpu())
        losses = []
        for slot, cid in enumerate(mine):
            tr.set_id(int(cid))
            tr.set_model_params(copy.deepcopy(glob))
            out = tr.train(self.dataset[5][int(cid)], self.device, self.args)
            if isinstance(out, (int, float)):
                losses.append(float(out))
            sd = tr.get_model_params()
            self.engine.set_client_params(slot, self.layout.flatten(sd, device=self.device))
        self.engine.last_loss = torch.tensor(sum(losses) / len(losses) if losses else float("nan"))

    def _robust_preaggregate(self, w):
        dt = getattr(self.args, "defense_type", None)
        if dt in ("norm_diff_clipping", "weak_dp"):
            mask = self.layout.weight_mask(self.device)
            ops.norm_diff_clip_(self.engine.params, self.global_flat, float(self.args.norm_bound), mask=mask)

    def _post_aggregate(self):
        if getattr(self.args, "defense_type", None) == "weak_dp":
            mask = self.layout.weight_mask(self.device)
            ops.gaussian_noise_(self.global_flat, float(self.args.stddev), seed=int(getattr(self.args, "random_seed", 0)),
                                offset=self.round_idx * self.layout.size, mask=mask)

    def close(self):
        self.engine.close()

    def run(self, rounds: Optional[int] = None):
        n = int(self.args.comm_round) if rounds is None else int(rounds)
        freq = int(getattr(self.args, "frequency_of_the_test", 0) or 0)
        for r in range(n):
            t0 = time.perf_counter()
            self._run_round_elastic(self.round_idx)
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            dt = time.perf_counter() - t0
            self.round_times.append(dt)
            rec = {"round_time_s": dt, "train_loss": float(self.engine.last_loss)}
            # GPU time per phase (HIP events, resolved after the round's synchronize)
            rec.update({f"gpu_ms/{k}": round(v, 3) for k, v in tracer().gpu_times().items()})
            # the SP simulator's schedule (reference fedavg_api.py:120-131): every ``frequency_of_the_test``-th
            # round and the last one
            last = self.round_idx == int(self.args.comm_round) - 1
            if (freq > 0 and self.round_idx % freq == 0) or last:
                t1 = time.perf_counter()
                rec.update(self.evaluate())
                if self.device.type == "cuda":
                    torch.cuda.synchronize(self.device)
                rec["eval_time_s"] = time.perf_counter() - t1
            self.history[self.round_idx] = rec
            if self.rank == 0:
                from ..common import scalar_metrics
                logging.info("[RCCL-sim] round %d: %s", self.round_idx, scalar_metrics(rec))
                MLOpsMetrics.get_instance().log(dict(scalar_metrics(rec), round=self.round_idx), step=self.round_idx)
            ck = getattr(self.args, "checkpoint_dir", None)
            if ck and (self.round_idx + 1) % int(getattr(self.args, "checkpoint_every", 1) or 1) == 0:
                self.save_checkpoint(ck)
            self.round_idx += 1
        # the final global model as a state dict, copied to the host only if the caller reads it (a device
        # snapshot is taken now: a bench loop that ignores the return value pays no host transfer)
        return _LazyState(self.layout, self.global_flat.detach().clone())

    def _run_round_elastic(self, round_idx):
        if not self.elastic:
            return self.run_round(round_idx)
        max_reinit = int(getattr(self.args, "elastic_max_reinit", 3) or 3)
        while True:
            try:
                return self.run_round(round_idx)
            except (RuntimeError, torch.distributed.DistBackendError) as e:
                from ...parallel import elastic
                # only a failed collective (a dead / unreachable peer) is retried, at most max_reinit times
                # per run; a local error (kernel fault, OOM, shape bug) would recur on every retry
                if not _is_peer_failure(e) or len(self.world_changes) >= max_reinit:
                    raise
                logging.warning("round %d: collective failed (%s) — re-initialising the communicator", round_idx,
                                str(e).splitlines()[0][:200])
                old = self.world
                self.rank, self.world = elastic.reinit(float(getattr(self.args, "elastic_settle_s", 3.0) or 3.0))
                self.world_changes.append((round_idx, old, self.world))
                self.C = math.ceil(self.K / self.world)
                if self.C != self.engine.C:   # more clients per rank now: a wider client stack
                    self.engine.close()
                    self.engine = ClientBatchEngine(self.model, self.C, self.device, self.args, self.compute_dtype)
                comm.broadcast_flat(self.global_flat, 0)   # every survivor restarts the round from rank 0's model

    # ---------------------------------------------------------------------------------------------
    def global_model_state(self):
        return self.layout.unflatten(self.global_flat.detach().cpu())

    @torch.no_grad()
    def evaluate(self, local_tests: bool = True):
        """The fork's per-round metrics of the global model (``evaluation.SimEvaluator``): ``Global/Acc``,
        ``Global/Loss``, ``Global/Recall`` of ``target_label`` on the rank-sharded global test set and, with
        ``local_tests``, ``_local_test_on_all_clients`` (every client's train and test data: federation accuracy /
        loss and per-client accuracy, recall and precision), all from one flat statistics buffer and one
        all-reduce. Task losses other than classification CE keep the global-test Acc / Loss below."""
        if self.dataset is None:
            return {}
        if self.engine.loss_name == "ce":
            if getattr(self, "_evaluator", None) is None:
                from .evaluation import SimEvaluator
                self._evaluator = SimEvaluator(self)
            return self._evaluator.evaluate(self.global_flat, local_tests=local_tests)
        test = self.dataset[3]
        self.model.load_state_dict(self.layout.unflatten(self.global_flat))
        self.model.eval()
        n = test.num_samples
        per = math.ceil(n / self.world)
        lo, hi = self.rank * per, min(n, (self.rank + 1) * per)
        stats = torch.zeros(3, device=self.device, dtype=torch.float32)
        bs = 512
        for s in range(lo, hi, bs):
            e = min(hi, s + bs)
            x = test.x[s:e].to(self.device)
            y = test.y[s:e].to(self.device)
            out = self.model(x).float()
            ln = self.engine.loss_name
            if ln == "nwp_ce":   # my_model_trainer_nwp.py test(): accuracy over non-padding tokens
                tok = y != 0
                stats[0] += ((out.argmax(1) == y) & tok).sum()
                stats[1] += torch.nn.functional.cross_entropy(out, y, ignore_index=0, reduction="sum")
                stats[2] += tok.sum()
            elif ln == "bce_sum":   # my_model_trainer_tag_prediction.py test(): exact tag-set match
                stats[0] += ((out > 0.5).int() == y.int()).all(1).sum()
                stats[1] += torch.nn.functional.binary_cross_entropy(out, y.float(), reduction="sum")
                stats[2] += (e - s)
            else:
                stats[0] += (out.argmax(-1) == y).sum()
                stats[1] += torch.nn.functional.cross_entropy(out, y, reduction="sum")
                stats[2] += (e - s)
        comm.all_reduce_flat(stats)
        self.model.train()
        tot = max(1.0, float(stats[2]))
        return {"Test/Acc": float(stats[0]) / tot, "Test/Loss": float(stats[1]) / tot}

    def save_checkpoint(self, directory):
        from ...core.checkpoint import save_round_checkpoint
        # per-run state beyond the global model: the clients' error-feedback residuals of compressed
        # updates (gathered from their owning ranks — every rank takes part). Data order and
        # augmentation are keyed by (seed, round, client), so the round index alone resumes them exactly
        # at any world size; the legacy generator state is kept for readers of the checkpoint layout.
        dense = self.residual.dense(self.K_total) if self.residual is not None else None
        if self.rank == 0:
            clients = {"gen": self.gen.get_state()}
            if dense is not None:
                clients["residual"] = dense.detach().cpu()
            if self.nova_buf is not None and not self.nova_first and self.nova_persist:
                clients["fednova_buf"] = self.nova_buf.detach().cpu()
            save_round_checkpoint(directory, self.round_idx, self.global_model_state(), self.args,
                                  server_opt=self.server_opt.state_dict() if self.server_opt else None,
                                  clients=clients)

    def load_checkpoint(self, directory, round_idx=None):
        from ...core.checkpoint import load_round_checkpoint
        ck = load_round_checkpoint(directory, round_idx)
        self.global_flat.copy_(self.layout.flatten(ck["global"], device=self.device))
        if self.server_opt is not None and ck.get("server_opt") is not None:
            self.server_opt.load_state_dict(ck["server_opt"])
        cl = ck.get("clients") or {}
        if cl.get("fednova_buf") is not None and self.nova_buf is not None:
            self.nova_buf.copy_(cl["fednova_buf"].to(self.device))
            self.nova_first = False
        if cl.get("gen") is not None and self.world == 1:
            self.gen.set_state(cl["gen"])
        if cl.get("residual") is not None and self.residual is not None:
            # rows go to the rank that trains each client in the resumed round
            self.assignment(int(ck["round"]) + 1)
            self.residual.load_dense(cl["residual"], self.round_owner)
        self.round_idx = int(ck["round"]) + 1
        return self.round_idx


class _ServerOptState:
    """FedOpt server optimizer on the flat global model (fused HIP kernel `fa_fedopt_step`)."""

    def __init__(self, args, P, device):
        self.opt = str(getattr(args, "server_optimizer", "sgd")).lower()
        self.lr = float(getattr(args, "server_lr", 1.0))
        self.momentum = float(getattr(args, "server_momentum", 0.0) or 0.0)
        self.b1 = float(getattr(args, "server_beta1", 0.9))
        self.b2 = float(getattr(args, "server_beta2", 0.99))
        self.eps = float(getattr(args, "server_eps", 1e-3))
        self.s1 = torch.zeros(P, device=device)
        self.s2 = torch.zeros(P, device=device)
        if self.opt in ("adagrad", "fedadagrad"):
            self.s2.fill_(float(getattr(args, "server_tau", 0.0)) ** 2)
        self.t = 0

    def step(self, glob, avg):
        self.t += 1
        ops.fedopt_step(avg.view(1, -1), torch.ones(1, device=avg.device), glob, self.opt, self.lr, self.b1, self.b2,
                        self.eps, self.momentum, False, self.s1, self.s2, self.t, first_step=self.t == 1)

    def state_dict(self):
        return {"s1": self.s1.cpu(), "s2": self.s2.cpu(), "t": self.t, "opt": self.opt}

    def load_state_dict(self, sd):
        self.s1.copy_(sd["s1"])
        self.s2.copy_(sd["s2"])
        self.t = int(sd["t"])
