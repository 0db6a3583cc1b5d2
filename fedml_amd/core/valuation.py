"""Client valuation (Shapley-style) for S-FedAvg / HS-FedAvg
(reference: `single_process/s_fedavg/fedavg_api.py:196-325`, `hs_fedavg/fedavg_api.py:177-230`).

The reference evaluates every coalition model one at a time: deep-copy the trainer, aggregate
the subset's state dicts in Python, run the validation loader — ``2·(2^(K-1)−1)·K + K``
aggregate+evaluate pairs per round for K clients. Here:

1. every distinct coalition is aggregated ONCE: the sample-weighted coalition averages are one
   ``[S, K] @ [K, P]`` product (``ops.subset_aggregate`` — fp32 MFMA kernel on MI355X);
2. the coalition models are evaluated TOGETHER: ``BatchedModelEvaluator`` runs up to
   ``max_models`` of them as one client-batched forward (grouped conv / bmm through
   ``parallel.batched_nn``) over the shared validation set;
3. the per-client values are then table lookups over the coalition scores ``v[mask]``.

So the reference's 2^(K-1)·2K evaluations become 2^K − 1, executed in ⌈(2^K−1)/max_models⌉
batched passes.
"""
import itertools
import logging
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from .. import ops
from .arena import ParamLayout


class BatchedModelEvaluator:
    def __init__(self, model: torch.nn.Module, device, max_models: int = 32, compute_dtype=None):
        self.model = model
        self.device = torch.device(device)
        self.layout = ParamLayout.from_module(model)
        self.max_models = max_models
        self.compute_dtype = compute_dtype
        self._interps = {}
        self._batched_ok = True
        self._native = {}            # chunk size → NativeResNetStep used for inference (GPU, CIFAR ResNets)
        self.native_images = 512     # images per model per native call (batches merged up to this)
        self._native_ok = self.device.type == "cuda"

    def flatten(self, state_dict) -> torch.Tensor:
        return self.layout.flatten(state_dict, device=self.device)

    def _interp(self, c):
        from ..parallel.batched_nn import BatchedInterpreter
        if c not in self._interps:
            self._interps[c] = BatchedInterpreter(self.model, self.layout, c)
        return self._interps[c]

    @torch.no_grad()
    def evaluate(self, flats: torch.Tensor, data, target_label: Optional[int] = None) -> Dict[str, torch.Tensor]:
        """flats: [S, P] models in this layout; data: iterable of (x, y). Returns per-model
        ``correct``, ``loss`` (sum), ``total`` and, with ``target_label``, ``tp``/``fp``/``fn``."""
        S = flats.shape[0]
        res = {k: torch.zeros(S, dtype=torch.float64) for k in ("correct", "loss", "tp", "fp", "fn")}
        total = 0
        batches = [(x.to(self.device), y.to(self.device)) for x, y in data]
        for y in (b[1] for b in batches):
            total += y.numel()
        for lo in range(0, S, self.max_models):
            chunk = flats[lo:lo + self.max_models].to(self.device)
            outs = self._run_chunk(chunk, batches)
            for k, v in self._score(outs, batches, target_label).items():
                res[k][lo:lo + chunk.shape[0]] = v.double().cpu()
        res["total"] = torch.full((S,), float(total), dtype=torch.float64)
        return res

    def _native_step(self, c):
        """The native HIP ResNet forward for ``c`` models at once (``NativeResNetStep.forward_eval``: the training
        kernels with BatchNorm folded from each model's running statistics), or None for other models."""
        if not self._native_ok:
            return None
        st = self._native.get(c)
        if st is None:
            from ..parallel.native_resnet import NativeResNetStep, UnsupportedNative
            try:
                st = NativeResNetStep(self.model, self.layout, c, self.device,
                                      dtype=self.compute_dtype or torch.float32, eval_only=True)
            except UnsupportedNative as e:
                logging.info("coalition evaluation: no native inference (%s)", e)
                self._native_ok = False
                return None
            self._native[c] = st
        return st

    def _bucket(self, c):
        """Model-stack width of the native step for a chunk of ``c`` models: the next power of two ≥ max(8, c),
        capped at ``max_models`` — small evaluations (the K singletons, a rank's shard of a sharded batch,
        Monte-Carlo prefixes) do not run ``max_models`` models, and only a handful of widths (each with its own
        native step and buffers) ever exist."""
        b = 8
        while b < c:
            b *= 2
        return max(c, min(b, self.max_models))

    def _run_chunk(self, chunk, batches):
        c = chunk.shape[0]
        cm = self._bucket(c)
        st = self._native_step(cm)
        if st is not None:
            # one native step (one set of buffers) per width bucket: a chunk narrower than its bucket is padded with
            # copies of its first model, whose outputs are dropped
            arena = chunk if c == cm else torch.cat([chunk, chunk[:1].expand(cm - c, -1)])
            arena = arena.contiguous()
            token = object()   # the calls after the first reuse this chunk's packed weights and folded BNs
            # consecutive batches run as one call of up to native_images images per model (an eval-only step
            # stores two activation buffers, so larger calls fit); the logits are split back per batch
            outs = []
            cap = self.native_images if getattr(st, "lean", False) else 0
            i = 0
            while i < len(batches):
                j, n = i + 1, batches[i][0].shape[0]
                while j < len(batches) and n + batches[j][0].shape[0] <= cap:
                    n += batches[j][0].shape[0]
                    j += 1
                x = batches[i][0] if j == i + 1 else torch.cat([b[0] for b in batches[i:j]])
                z = st.forward_eval(arena, x.unsqueeze(0).expand(cm, *x.shape), models_token=token)[:c].float()
                outs.extend(z.split([b[0].shape[0] for b in batches[i:j]], dim=1))
                i = j
            return outs
        if self._batched_ok:
            try:
                interp = self._interp(c)
                views = {s.key: chunk[:, s.offset:s.offset + s.numel].view(c, *s.shape) for s in self.layout.slots}
                return [interp.run(views, x.unsqueeze(0).expand(c, *x.shape).contiguous(), training=False,
                                   dtype=self.compute_dtype).float() for x, _ in batches]
            except Exception as e:  # models the fx tracer cannot batch → sequential functional calls
                logging.info("batched evaluation unavailable (%s); evaluating models sequentially", e)
                self._batched_ok = False
        outs = [[] for _ in batches]
        for i in range(c):
            sd = self.layout.unflatten(chunk[i])
            params = {k: v.to(self.device) for k, v in sd.items()}
            self.model.to(self.device).eval()
            for bi, (x, _) in enumerate(batches):
                outs[bi].append(torch.func.functional_call(self.model, params, (x,)).float())
        return [torch.stack(o) for o in outs]

    @staticmethod
    def _score(outs, batches, target_label):
        c = outs[0].shape[0]
        acc = {k: torch.zeros(c, device=outs[0].device) for k in ("correct", "loss", "tp", "fp", "fn")}
        for out, (_, y) in zip(outs, batches):
            pred = out.argmax(-1)
            yy = y.unsqueeze(0).expand_as(pred)
            acc["correct"] += (pred == yy).sum(1)
            acc["loss"] += torch.nn.functional.cross_entropy(out.reshape(-1, out.shape[-1]), yy.reshape(-1),
                                                             reduction="none").view(c, -1).sum(1)
            if target_label is not None:
                t = int(target_label)
                acc["tp"] += ((pred == t) & (yy == t)).sum(1)
                acc["fp"] += ((pred == t) & (yy != t)).sum(1)
                acc["fn"] += ((pred != t) & (yy == t)).sum(1)
        return acc


def coalition_weights(masks: Sequence[int], sample_nums: Sequence[float]) -> torch.Tensor:
    """[S, K] sample-weighted averaging matrix for coalitions given as bitmasks."""
    K = len(sample_nums)
    n = torch.tensor([float(v) for v in sample_nums], dtype=torch.float64)
    W = torch.zeros(len(masks), K, dtype=torch.float64)
    for r, m in enumerate(masks):
        sel = torch.tensor([(m >> k) & 1 for k in range(K)], dtype=torch.bool)
        W[r, sel] = n[sel] / n[sel].sum()
    return W.float()


def score_from_metrics(m: Dict[str, torch.Tensor], score: str = "acc", target_label=None) -> torch.Tensor:
    """Per-model score used as the coalition value: accuracy or target-label F1/recall/precision."""
    if target_label is None or score.lower() in ("acc", "accuracy"):
        return m["correct"] / m["total"].clamp_min(1)
    tp, fp, fn = m["tp"], m["fp"], m["fn"]
    s = score.lower()
    if s == "f1":
        return torch.where(2 * tp + fp + fn > 0, 2 * tp / (2 * tp + fp + fn).clamp_min(1e-12), torch.zeros_like(tp))
    if s in ("sensitivity", "recall", "tpr"):
        return torch.where(tp + fn > 0, tp / (tp + fn).clamp_min(1e-12), torch.zeros_like(tp))
    if s in ("precision", "ppv"):
        return torch.where(tp + fp > 0, tp / (tp + fp).clamp_min(1e-12), torch.zeros_like(tp))
    return m["correct"] / m["total"].clamp_min(1)


class CoalitionValuer:
    """Caches coalition values v(mask) for one round's K local models."""

    _METRICS = ("correct", "loss", "tp", "fp", "fn", "total")

    def __init__(self, evaluator: BatchedModelEvaluator, flats: torch.Tensor, sample_nums, valid_data,
                 score="acc", target_label=None, shard: bool = False):
        """``shard``: every rank of the process group evaluates its share of each batch of new coalitions
        (coalition i of the sorted batch on rank i mod W) and the scores are all-gathered — the coalition
        evaluation spreads over the GPUs (all ranks must call ``ensure`` with the same masks)."""
        self.ev = evaluator
        self.flats = flats.to(evaluator.device)
        self.n = list(sample_nums)
        self.K = len(self.n)
        self.data = list(valid_data)
        self.score = score
        self.target = target_label
        self.v: Dict[int, float] = {0: 0.0}
        self.metrics: Dict[int, Dict[str, float]] = {}
        self.evaluations = 0
        from ..parallel import comm
        self._comm = comm
        self.shard = bool(shard) and comm.is_dist()

    def ensure(self, masks: Sequence[int]):
        todo = sorted({m for m in masks if m not in self.v})
        if not todo:
            return
        if self.shard:
            m = self._sharded_metrics(todo)
        else:
            W = coalition_weights(todo, self.n).to(self.flats.device)
            m = self.ev.evaluate(ops.subset_aggregate(W, self.flats), self.data, self.target)
        vals = score_from_metrics(m, self.score, self.target)
        for i, mask in enumerate(todo):
            self.v[mask] = float(vals[i])
            self.metrics[mask] = {k: float(t[i]) for k, t in m.items()}
        self.evaluations += len(todo)

    def _sharded_metrics(self, todo):
        comm = self._comm
        R, r = comm.world_size(), comm.rank()
        mine = todo[r::R]
        per = -(-len(todo) // R)
        packed = torch.zeros(per, len(self._METRICS), dtype=torch.float64, device=self.flats.device)
        if mine:
            W = coalition_weights(mine, self.n).to(self.flats.device)
            m = self.ev.evaluate(ops.subset_aggregate(W, self.flats), self.data, self.target)
            packed[:len(mine)] = torch.stack([m[k] for k in self._METRICS], 1).to(packed.device)
        parts = comm.all_gather_flat(packed.view(-1))
        out = torch.zeros(len(todo), len(self._METRICS), dtype=torch.float64)
        for q, part in enumerate(parts):
            n_q = len(todo[q::R])
            out[q::R] = part.view(per, -1)[:n_q].cpu()
        return {k: out[:, j].clone() for j, k in enumerate(self._METRICS)}

    def exact_reference_sv(self) -> List[float]:
        """The reference's exact estimator: for client i, average over every non-empty coalition
        S of the others of [v(S ∪ i) − v(S)], plus v({i}) as one more term (accuracy deltas are
        normalised by the partial model's total, identical to accuracy differences here)."""
        K = self.K
        full = (1 << K) - 1
        self.ensure(range(1, full + 1))
        sv = []
        for i in range(K):
            bit = 1 << i
            ap, cnt = 0.0, 0
            for S in range(1, full + 1):
                if S & bit:
                    continue
                ap += self.v[S | bit] - self.v[S]
                cnt += 1
            ap += self.v[bit]
            cnt += 1
            sv.append(ap / cnt)
        return sv

    def monte_carlo_sv(self, rng: np.random.RandomState, tol=0.005, max_perms=None, batch_perms=None) -> List[float]:
        """Permutation-sampling Shapley values (Castro et al.): average marginal contribution of
        each client over random orderings; stops when the last three SV updates moved < ``tol``
        (Euclidean) or after K² permutations — the reference's stopping rule. Unlike the reference
        (which shuffles but then evaluates the UNshuffled prefixes), marginals are
        credited to the permuted client. Prefix coalitions of a batch of permutations are
        evaluated together."""
        K = self.K
        max_perms = max_perms or K * K
        batch_perms = batch_perms or max(1, K)
        sv = np.zeros(K)
        d: List[float] = []
        done = 0
        while True:
            perms = [rng.permutation(K) for _ in range(min(batch_perms, max_perms - done))]
            prefixes = []
            for p in perms:
                m = 0
                for c in p:
                    m |= 1 << int(c)
                    prefixes.append(m)
            self.ensure(prefixes)
            for p in perms:
                last = sv.copy()
                m, prev = 0, 0.0
                contrib = np.zeros(K)
                for c in p:
                    m |= 1 << int(c)
                    contrib[int(c)] = self.v[m] - prev
                    prev = self.v[m]
                sv = (done * sv + contrib) / (done + 1)
                if done:
                    d.append(float(np.linalg.norm(sv - last)))
                done += 1
            if done >= max_perms:
                break
            if done > K and all(x < tol for x in d[-3:]):
                break
        return sv.tolist()
