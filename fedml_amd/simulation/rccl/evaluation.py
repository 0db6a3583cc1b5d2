"""Evaluation for the RCCL simulator: the fork's per-round metrics, computed on the device and all-reduced.

Reference (sequential, host-side counting per batch):
  * `single_process/fedavg/fedavg_api.py:130-177` — ``Global/Acc`` and ``Global/Recall`` (sklearn ``recall_score`` of
    ``target_label``) of the global model on the global test set, every evaluated round;
  * `:238-326` ``_local_test_on_all_clients`` — the global model on EVERY client's train and test data: federation
    accuracy / loss plus per-client accuracy and per-class recall / precision lists;
  * `my_model_trainer_classification.py:113-154` — the per-class recall / precision formula.

Here every sample is evaluated once by the global model: the samples of this rank's share (global test rows split
into contiguous ranges per rank; clients ``c ≡ rank (mod world)`` for the local tests) run through the native HIP
ResNet forward (``NativeResNetStep.forward_eval`` with the global model in every row of a small model stack, i.e.
one wide batch per launch sequence) or the torch module, and one K8b kernel pass per logits block
(``ops.eval_stats``: argmax, cross-entropy, per-client true-positive / actual / predicted class counts) accumulates
straight into one flat statistics buffer. One all-reduce of that buffer gives every rank the whole federation's
numbers; the per-client dicts are then formed on the host (``simulation.common``).
"""
import math
from typing import Dict, Optional

import torch

from ... import ops
from ...parallel import comm
from ..common import class_rates, fork_local_test_stats

# native inference geometry: the global model replicated in ``_ROWS`` arena rows, each row a batch of up to ``_N_MAX``
# images (``_ROWS`` × ``_N_MAX`` = 6400 images per forward, the training step's width at the headline geometry)
_ROWS = 16
_N_MAX = 400


def _num_classes(model: torch.nn.Module, dataset) -> int:
    if dataset is not None and len(dataset) > 7 and dataset[7]:
        return int(dataset[7])
    last = [m for m in model.modules() if isinstance(m, torch.nn.Linear)]
    return int(last[-1].out_features) if last else 1


class SimEvaluator:
    """Global-model evaluation of an ``RCCLSimulator`` (all ranks call ``evaluate`` together)."""

    def __init__(self, sim):
        self.sim = sim
        self.device = sim.device
        self.K = _num_classes(sim.model, sim.dataset)
        ds = sim.dataset
        self.target = None
        if ds is not None and len(ds) > 8 and ds[8] is not None:
            self.target = int(ds[8])
        elif getattr(sim.args, "target_label", None) is not None:
            self.target = int(sim.args.target_label)
        self._native = None          # NativeResNetStep for inference (None: not built yet, False: unavailable)
        self._n_row = None
        self._global = None          # (x, y) of the global test set on the device
        self._test_store = None      # per-client test data on the device (DeviceClientStore)

    # ------------------------------------------------------------------------------------------ inference
    def _native_step(self):
        if self._native is None:
            self._native = False
            from ...parallel.native_resnet import NativeResNetStep
            st = self.sim.engine.native_step
            if type(st) is NativeResNetStep:
                self._native = NativeResNetStep(self.sim.model, self.sim.layout, _ROWS, self.device, dtype=st.dtype,
                                                eval_only=True)
        return self._native or None

    def _accumulate(self, flat, x_all, y_all, idx, groups, sums, cls):
        """Evaluate the global model ``flat`` on samples ``x_all[idx]`` and add their statistics into group rows
        ``groups`` of ``sums`` [G, 3] / ``cls`` [G, 3, K] (None: no class counts)."""
        n = int(idx.numel())
        if n == 0:
            return
        st = self._native_step()
        if st is not None:
            if self._n_row is None:      # one inference geometry for every later call (last chunk zero-padded)
                self._n_row = min(_N_MAX, max(8, 8 * math.ceil(n / (_ROWS * 8))))
            cap = _ROWS * self._n_row
            arena = flat.view(1, -1).expand(_ROWS, -1).contiguous()
            token = object()   # one model for every chunk: packed weights and BN folds once per call
            for lo in range(0, n, cap):
                hi = min(n, lo + cap)
                sel = idx[lo:hi]
                x = x_all[sel].to(torch.float32)
                y = y_all[sel].reshape(-1)
                g = groups[lo:hi]
                if hi - lo < cap:
                    pad = cap - (hi - lo)
                    x = torch.cat([x, x.new_zeros((pad,) + tuple(x.shape[1:]))])
                    y = torch.cat([y, y.new_full((pad,), -1)])
                    g = torch.cat([g, g.new_full((pad,), -1)])
                logits = st.forward_eval(arena, x.view(_ROWS, self._n_row, *x.shape[1:]),
                                         models_token=token).reshape(cap, -1)
                ops.eval_stats(logits, y, g, sums=sums, cls=cls, with_classes=cls is not None)
            return
        model = self.sim.model
        model.load_state_dict(self.sim.layout.unflatten(flat))
        model.eval()
        bs = 512
        for lo in range(0, n, bs):
            sel = idx[lo:lo + bs]
            out = model(x_all[sel]).float()
            out = out.reshape(out.shape[0], -1)
            ops.eval_stats(out, y_all[sel].reshape(-1), groups[lo:lo + bs], sums=sums, cls=cls,
                           with_classes=cls is not None)
        model.train()

    # ------------------------------------------------------------------------------------------ data
    def _global_data(self):
        if self._global is None:
            test = self.sim.dataset[3]
            if test is None:            # no global test split: the Global/* metrics are None
                self._global = (None, torch.zeros(0, dtype=torch.int64, device=self.device))
            else:
                self._global = (test.x.to(self.device), test.y.to(self.device))
        return self._global

    def _client_test_store(self):
        if self._test_store is None:
            from .client_store import DeviceClientStore
            tl = self.sim.dataset[6]
            have = {c: d for c, d in tl.items() if d is not None}
            self._test_store = (DeviceClientStore.from_client_data(have, self.device) if have else None, sorted(have))
        return self._test_store

    @staticmethod
    def _client_rows(store, pos_of, clients, device):
        """Sample indices of ``clients`` in ``store`` (``pos_of[c]``: the client's position in it) and the
        client id of each row."""
        idx, grp = [], []
        for c in clients:
            p = pos_of.get(c)
            if p is None:
                continue
            o, n = int(store.offsets[p]), store.counts_host[p]
            idx.append(torch.arange(o, o + n, device=device))
            grp.append(torch.full((n,), int(c), dtype=torch.int32, device=device))
        if not idx:
            return torch.zeros(0, dtype=torch.int64, device=device), torch.zeros(0, dtype=torch.int32, device=device)
        return torch.cat(idx), torch.cat(grp)

    # ------------------------------------------------------------------------------------------ metrics
    @torch.no_grad()
    def evaluate(self, flat: torch.Tensor, local_tests: bool = True) -> Dict[str, object]:
        sim, K, dev = self.sim, self.K, self.device
        rank, world = sim.rank, sim.world
        Kt = sim.K_total
        # one flat buffer: global (3 + 3K) | train sums [Kt, 3] | test sums [Kt, 3] | test classes [Kt, 3, K]
        nG = 3 + 3 * K
        nL = (6 + 3 * K) * Kt if local_tests else 0
        buf = torch.zeros(nG + nL, dtype=torch.float32, device=dev)
        g_sums = buf[:3].view(1, 3)
        g_cls = torch.zeros(1, 3, K, dtype=torch.int32, device=dev)
        x, y = self._global_data()
        per = math.ceil(len(y) / world)
        lo, hi = rank * per, min(len(y), (rank + 1) * per)
        rows = torch.arange(lo, max(lo, hi), device=dev)
        self._accumulate(flat, x, y, rows, torch.zeros(len(rows), dtype=torch.int32, device=dev), g_sums, g_cls)
        buf[3:nG].copy_(g_cls.view(-1).to(torch.float32))
        if local_tests:
            tr_sums = buf[nG:nG + 3 * Kt].view(Kt, 3)
            te_sums = buf[nG + 3 * Kt:nG + 6 * Kt].view(Kt, 3)
            te_cls = torch.zeros(Kt, 3, K, dtype=torch.int32, device=dev)
            tstore, tclients = self._client_test_store()
            mine = [c for c in tclients if c % world == rank]      # the reference skips clients without test data
            idx, grp = self._client_rows(sim.store, {c: c for c in range(sim.store.num_clients)}, mine, dev)
            self._accumulate(flat, sim.store.x_all, sim.store.y_all, idx, grp, tr_sums, None)
            if tstore is not None:
                idx, grp = self._client_rows(tstore, {c: p for p, c in enumerate(tclients)}, mine, dev)
                self._accumulate(flat, tstore.x_all, tstore.y_all, idx, grp, te_sums, te_cls)
            buf[nG + 6 * Kt:].copy_(te_cls.view(-1).to(torch.float32))
        comm.all_reduce_flat(buf)
        h = buf.double().cpu()
        gs, gc = h[:3], h[3:nG].view(3, K)
        out: Dict[str, object] = {}
        if local_tests:
            trs, tes = h[nG:nG + 3 * Kt].view(Kt, 3), h[nG + 3 * Kt:nG + 6 * Kt].view(Kt, 3)
            tec = h[nG + 6 * Kt:].view(Kt, 3, K)
            train_m, test_m = [], []
            for c in self._client_test_store()[1]:
                train_m.append({"test_correct": float(trs[c, 0]), "test_loss": float(trs[c, 1]),
                                "test_total": int(trs[c, 2])})
                rec, prec = class_rates(tec[c, 0], tec[c, 1], tec[c, 2])
                test_m.append({"test_correct": float(tes[c, 0]), "test_loss": float(tes[c, 1]),
                               "test_total": int(tes[c, 2]), "test_recall": rec, "test_precision": prec})
            out.update(fork_local_test_stats(train_m, test_m))
        if float(gs[2]) == 0:
            out.update({"Global/Acc": None, "Global/Loss": None, "Global/Recall": None})
            return out
        tot = float(gs[2])
        out["Global/Acc"] = float(gs[0]) / tot
        out["Global/Loss"] = float(gs[1]) / tot
        recall: Optional[float] = None
        if self.target is not None and 0 <= self.target < K:
            act = float(gc[1, self.target])
            recall = float(gc[0, self.target]) / act if act > 0 else 0.0   # sklearn recall_score (zero_division=0)
        out["Global/Recall"] = recall
        return out
