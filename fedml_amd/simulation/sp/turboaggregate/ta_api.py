"""TurboAggregate, sequential (reference: `single_process/turboaggregate/TA_trainer.py:12-206` —
plain FedAvg with an unused MPC library). Here every round's aggregation runs the SecAgg
protocol of ``core.mpc`` in-process: each sampled client uploads
``Q(n_c/N · w_c) + pairwise masks (mod p)``; clients listed in
``args.ta_dropout_ranks[round]`` (0-based positions in the round) drop after key exchange and
their masks are removed through Shamir (BGW) reconstruction from ``T+1`` survivors. Integer
buffers are carried from the first survivor. ``ta_secure: false`` degrades to plain FedAvg."""
import copy
import time

import torch

from ....core.mpc import SecAggClient, SecureAggregator
from ....core.mpc.finite_field import DEFAULT_PRIME
from ..fedavg.fedavg_api import FedAvgAPI
from ...mp.turboaggregate import flatten_float, unflatten_float


class TurboAggregateAPI(FedAvgAPI):
    def __init__(self, args, device, dataset, model, model_trainer=None):
        super().__init__(args, device, dataset, model, model_trainer)
        self.secure = bool(getattr(args, "ta_secure", True))
        self.frac_bits = int(getattr(args, "ta_frac_bits", 20))
        self._round = 0
        self.dropped_history = []

    def _aggregate(self, w_locals):
        if not self.secure:
            return super()._aggregate(w_locals)
        K = len(w_locals)
        T = int(getattr(self.args, "ta_threshold", max(1, K // 2)))
        drops = getattr(self.args, "ta_dropout_ranks", None) or {}
        dropped = set(int(d) for d in drops.get(self._round, drops.get(str(self._round), [])))
        n_total = float(sum(n for n, _ in w_locals))
        dev = self.device if self.device is not None else torch.device("cpu")
        clients = [SecAggClient(i, K, T, DEFAULT_PRIME, self.frac_bits, seed=(self._round << 16) + i) for i in range(K)]
        sa = SecureAggregator(K, T, DEFAULT_PRIME, self.frac_bits)
        for c in clients:
            sa.add_public_key(c.cid, c.pk)
        for c in clients:
            for holder, share in enumerate(c.sk_shares()):
                sa.add_share(c.cid, holder, share)
        masked = {}
        for i, (n, w) in enumerate(w_locals):
            if i in dropped:
                continue
            masked[i] = clients[i].masked_input(flatten_float(w).to(dev) * (float(n) / n_total), sa.pks)
        avg = sa.aggregate(masked)
        alive_mass = sum(float(w_locals[i][0]) for i in masked)
        avg = avg * (n_total / alive_mass)
        self.dropped_history.append(sorted(dropped))
        self._round += 1
        return unflatten_float(avg.cpu(), w_locals[min(masked)][1])

    aggregate = _aggregate
