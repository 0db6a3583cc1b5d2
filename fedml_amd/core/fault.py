"""Failure injection for FL rounds.

The reference has no elastic recovery: every server waits for all selected clients
(`FedAVGAggregator.py:59-66`, `cross_silo/horizontal/fedml_server_manager.py:121-207`) and the only
injected faults are adversarial (backdoor attackers). Here a round can lose clients:

* ``client_dropout_prob`` — a selected client trains but its upload never arrives;
* ``client_delay_mean`` (seconds, ``client_delay_dist`` = ``exp`` | ``const``) — simulated upload delay;
  with ``round_deadline`` (seconds) a client whose delay exceeds it misses the round;
* ``client_dropout_ids`` — clients that never upload (a dead silo);
* ``fault_seed`` — the draws are a pure function of (seed, round, client id), so every rank and every
  re-run agrees on who dropped.

Servers aggregate whoever arrived, re-weighted by the survivors' sample counts (the RCCL simulator
zeroes the weights of lost clients; the cross-silo server closes a round at ``round_timeout``).
"""
import json

import numpy as np


class FaultInjector:
    def __init__(self, args=None, dropout_prob=None, delay_mean=None, delay_dist=None, deadline=None, seed=None):
        g = (lambda k, d: getattr(args, k, d) if args is not None else d)
        self.p = float(dropout_prob if dropout_prob is not None else (g("client_dropout_prob", 0.0) or 0.0))
        self.delay_mean = float(delay_mean if delay_mean is not None else (g("client_delay_mean", 0.0) or 0.0))
        self.dist = str(delay_dist if delay_dist is not None else (g("client_delay_dist", "exp") or "exp"))
        dl = deadline if deadline is not None else g("round_deadline", None)
        self.deadline = float(dl) if dl not in (None, "", 0, 0.0) else None
        self.seed = int(seed if seed is not None else (g("fault_seed", g("random_seed", 0)) or 0))
        ids = g("client_dropout_ids", None)
        if isinstance(ids, str):
            ids = json.loads(ids) if ids.strip() else []
        self.always = {int(i) for i in (ids or [])}

    @property
    def active(self) -> bool:
        return self.p > 0 or bool(self.always) or (self.delay_mean > 0 and self.deadline is not None)

    def _rng(self, round_idx, client_id):
        return np.random.default_rng([self.seed & 0xFFFFFFFF, int(round_idx), int(client_id), 0x5EED])

    def dropped(self, round_idx: int, client_id: int) -> bool:
        if int(client_id) in self.always:
            return True
        return self.p > 0 and self._rng(round_idx, client_id).random() < self.p

    def delay(self, round_idx: int, client_id: int) -> float:
        if self.delay_mean <= 0:
            return 0.0
        if self.dist == "const":
            return self.delay_mean
        r = self._rng(round_idx, client_id)
        r.random()                       # decorrelate from the dropout draw
        return float(r.exponential(self.delay_mean))

    def arrives(self, round_idx: int, client_id: int) -> bool:
        """True when the client's upload reaches the server before the round deadline."""
        if self.dropped(round_idx, client_id):
            return False
        return self.deadline is None or self.delay(round_idx, client_id) <= self.deadline

    def survivors(self, round_idx: int, client_ids) -> np.ndarray:
        return np.array([self.arrives(round_idx, c) for c in client_ids], dtype=bool)
