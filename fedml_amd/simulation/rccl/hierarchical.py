"""Hierarchical FL on the virtual-client engine (reference: `single_process/hierarchical_fl/trainer.py:1-115`,
`group.py:7-70`, `client.py`; sequential re-statement: `sp/hierarchical_fl/trainer.py`).

The reference trains every sampled client of every group one after another on one shared model (a ``deepcopy`` of
the group model per client), averages state dicts per group and global epoch in Python, then averages the groups.
Here one global round is:

  * every sampled client of every group trains AT ONCE in the client-batched engine (clients packed over the GPUs);
  * a group round's end is a two-level reduce: intra-GPU, the rank's client stack is reduced to per-group sums with
    ONE ``[G, C] × [C, P]`` MFMA product (``ops.subset_aggregate``: row g holds n_c for the rank's clients of group
    g); intra-node, one RCCL all-reduce of the ``[G, P + 1]`` buffer (sums ‖ sample totals) gives every rank every
    group model;
  * the next group round starts every client slot from its own group's model (one row gather ``params ←
    w_groups[group_of_slot]``);
  * the global model at any global epoch is Σ_g N_g·w_g / Σ_g N_g = Σ_c n_c·w_c / Σ_c n_c, read off the same
    buffer — no second collective.

Per-epoch group snapshots (what the reference keeps for its evaluation schedule) are reduced only at the epochs
``frequency_of_the_test`` evaluates and at each group round's end. Client sampling and the random group assignment
use the reference's generators (``np.random.seed(round)``; ``np.random.randint`` at construction — drawn on rank 0
and broadcast)."""
import logging
import time

import numpy as np
import torch

from ... import ops
from ...parallel import comm
from ..common import client_sampling
from .simulator import RCCLSimulator


class HierarchicalRCCLSimulator(RCCLSimulator):
    def __init__(self, args, device, dataset, model, store=None, model_trainer=None):
        super().__init__(args, device, dataset, model, store=store, model_trainer=model_trainer)
        method = str(getattr(args, "group_method", "random"))
        if method != "random":
            raise ValueError(f"group_method {method} not supported (reference supports 'random')")
        if self.compression or self.server_opt is not None or self.fednova or self.user_trainer is not None:
            raise ValueError("hierarchical FL on the RCCL engine: plain FedAvg groups only")
        self.G = int(getattr(args, "group_num", 1))
        gi = torch.as_tensor(np.random.randint(0, self.G, self.K_total), dtype=torch.int64, device=self.device)
        comm.broadcast_flat(gi, 0)
        self.group_indexes = gi.cpu().numpy()
        self.global_rounds = int(getattr(args, "global_comm_round", getattr(args, "comm_round", 1)))
        self.group_rounds = int(getattr(args, "group_comm_round", 1))
        self.E = int(args.epochs)
        self.hier_history = []
        self._gbuf = torch.empty(self.G, self.layout.size + 1, dtype=torch.float32, device=self.device)

    def group_client_sampling(self, global_round_idx):
        sampled = client_sampling(global_round_idx, self.K_total, self.K)
        out = {}
        for c in sampled:
            out.setdefault(int(self.group_indexes[c]), []).append(int(c))
        return out

    def _group_reduce(self, Wg):
        """[G, P + 1] = per-group Σ n_c·w_c ‖ Σ n_c over every rank's clients (one GEMM + one all-reduce)."""
        P = self.layout.size
        self._gbuf[:, :P].copy_(ops.subset_aggregate(Wg, self.engine.params))
        self._gbuf[:, P].copy_(Wg.sum(1))
        comm.all_reduce_flat(self._gbuf)
        return self._gbuf

    def _global_from(self, gbuf):
        P = self.layout.size
        tot = gbuf[:, P].sum().clamp_min(1e-12)
        return gbuf[:, :P].sum(0) / tot

    def run_global_round(self, gr: int):
        args = self.args
        ids, mine = self.assignment(gr)
        C, P = self.C, self.layout.size
        slots = torch.zeros(C, dtype=torch.int64)
        valid = torch.zeros(C, dtype=torch.bool)
        for i, cid in enumerate(mine):
            slots[i], valid[i] = cid, True
        gslot = torch.tensor([int(self.group_indexes[c]) for c in mine] + [0] * (C - len(mine)), dtype=torch.int64,
                             device=self.device)
        Wg = torch.zeros(self.G, C, dtype=torch.float32)
        for i, cid in enumerate(mine):
            Wg[int(self.group_indexes[cid]), i] = float(self.sample_counts[cid])
        Wg = Wg.to(self.device)
        slots, valid = slots.to(self.device), valid.to(self.device)
        freq = int(getattr(args, "frequency_of_the_test", 1) or 1)
        last_epoch = self.global_rounds * self.group_rounds * self.E - 1
        gbuf = None
        for r in range(self.group_rounds):
            if r == 0:
                self.engine.load_global(self.global_flat)
            else:
                w_groups = gbuf[:, :P] / gbuf[:, P:].clamp_min(1e-12)
                with torch.no_grad():
                    self.engine.params.copy_(w_groups.index_select(0, gslot))
                self.engine._shadow_stale = True
            for e in range(self.E):
                ge = (gr * self.group_rounds + r) * self.E + e
                rng_key = (int(getattr(args, "random_seed", 0)) * 1000003 + ge * 7919) & 0x7FFFFFFF
                self.engine.train(self.store, slots, 1, int(args.batch_size), float(args.learning_rate),
                                  generator=self.gen, shuffle=bool(getattr(args, "shuffle", True)), valid_slots=valid,
                                  rng_key=rng_key)
                evaluate = ge % freq == 0 or ge == last_epoch      # the SP trainer's schedule (freq 0 → every epoch)
                if e == self.E - 1 or evaluate:
                    gbuf = self._group_reduce(Wg)
                if evaluate and self.dataset is not None:
                    keep = self.global_flat.clone()
                    self.global_flat.copy_(self._global_from(gbuf))
                    stats = self.evaluate()
                    stats["global_epoch"] = ge
                    self.hier_history.append(stats)
                    self.global_flat.copy_(keep)
        self.global_flat.copy_(self._global_from(gbuf))

    def run(self, rounds=None):
        n = self.global_rounds if rounds is None else int(rounds)
        for _ in range(n):
            t0 = time.perf_counter()
            self.run_global_round(self.round_idx)
            if self.device.type == "cuda":
                torch.cuda.synchronize(self.device)
            dt = time.perf_counter() - t0
            self.round_times.append(dt)
            self.history[self.round_idx] = {"round_time_s": dt, "train_loss": float(self.engine.last_loss)}
            if self.rank == 0:
                logging.info("[RCCL-hier] global round %d: %.3fs", self.round_idx, dt)
            self.round_idx += 1
        return self.global_model_state()
