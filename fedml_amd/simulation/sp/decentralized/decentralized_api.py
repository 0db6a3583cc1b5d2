"""Decentralized online learning: DSGD ("DOL") and PushSum over a gossip topology
(reference: `single_process/decentralized/{decentralized_fl_api,client_dsgd,client_pushsum}.py`).

All N workers' parameters live in ONE ``[N, P]`` arena: an iteration computes every worker's
gradient on its current streaming sample with a vmapped functional call, takes the local step
``x ← x − η·∇f_i(z_i)``, and gossips with a single mixing product ``X ← Wᵀ X`` (sender-weighted
like the reference: worker j pushes ``W[j,i]·x_j`` to i). PushSum additionally mixes the weights
``ω ← Wᵀ ω`` and de-biases ``z = x / ω`` (needed for the row-stochastic asymmetric topology).
The reference hands every client the SAME model object (so its "workers" share parameters);
here each worker really has its own. ``mode: LOCAL`` trains without communication.
Regret = average loss over workers and iterations so far (reference ``cal_regret``).

Multi-GPU (one process per GPU, ``torch.distributed`` initialised — RCCL over xGMI): the N workers
are sharded over the ranks; each rank computes its workers' gradients and local steps, ONE
``all_gather`` of the gossip rows per iteration replaces the reference's per-neighbour sends
(``client_dsgd.py:104-122``), and each rank mixes only its own receiver rows ``X_own ← W[:, own]ᵀ X``
on the MFMA kernel. The result equals the single-process run (tests/test_decentralized_dist.py).
"""
import logging

import numpy as np
import torch
from torch.func import functional_call, grad, vmap

from ....core.distributed.topology import AsymmetricTopologyManager, SymmetricTopologyManager
from .... import ops
from ....parallel import comm


def _streams_from_dataset(dataset, n_clients):
    """Per-client streams [(x_t, y_t)] from the standard 8-tuple's local train sets."""
    train_local = dataset[5]
    xs, ys = [], []
    for c in range(n_clients):
        bx, by = [], []
        for x, y in train_local[c]:
            bx.append(x.reshape(x.shape[0], -1).float())
            by.append(y.reshape(-1))
        xs.append(torch.cat(bx))
        ys.append(torch.cat(by))
    T = min(len(x) for x in xs)
    return torch.stack([x[:T] for x in xs]), torch.stack([y[:T] for y in ys])


class DecentralizedFLAPI:
    def __init__(self, args, device, dataset, model, model_trainer=None):
        self.args = args
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.N = int(getattr(args, "client_num_in_total", 0) or getattr(args, "client_number", 0))
        if isinstance(dataset, tuple) and len(dataset) == 2 and torch.is_tensor(dataset[0]):
            self.X, self.Y = dataset  # [N, T, d], [N, T]
        else:
            self.X, self.Y = _streams_from_dataset(dataset, self.N)
        self.X, self.Y = self.X.to(self.device), self.Y.to(self.device)
        self.T = int(getattr(args, "iteration_number", self.X.shape[1]))
        self.mode = str(getattr(args, "mode", "DOL")).upper()
        self.lr = float(args.learning_rate)
        self.wd = float(getattr(args, "weight_decay", 0.0) or 0.0)
        self.epoch = int(getattr(args, "epoch", getattr(args, "epochs", 1)) or 1)
        sym = bool(getattr(args, "b_symmetric", True))
        k = int(getattr(args, "topology_neighbors_num_undirected", 2))
        if sym:
            self.topo = SymmetricTopologyManager(self.N, k)
        else:
            self.topo = AsymmetricTopologyManager(self.N, k, int(getattr(args, "topology_neighbors_num_directed", 2)))
        self.topo.generate_topology()
        self.mix = self.topo.mixing_matrix(self.device).t().contiguous()  # receiver-major: X ← Wᵀ X
        self.model = model.to(self.device)
        self.names = [n for n, _ in self.model.named_parameters()]
        self.shapes = [p.shape for _, p in self.model.named_parameters()]
        flat0 = torch.cat([p.detach().reshape(-1) for p in self.model.parameters()]).float()
        self.x = flat0.unsqueeze(0).repeat(self.N, 1)       # gossip variable
        self.omega = torch.ones(self.N, 1, device=self.device)
        self.z = self.x.clone()                              # de-biased model used for the loss
        self.regret_history = []
        # rank sharding of the workers (world 1: all rows local)
        self.rank, self.world = comm.rank(), comm.world_size()
        self.per = -(-self.N // self.world)
        if self.world > 1:   # one topology for all ranks (the generators draw random edges)
            comm.broadcast_flat(self.mix, 0)
        self.lo, self.hi = min(self.N, self.rank * self.per), min(self.N, (self.rank + 1) * self.per)
        out_dim = None
        with torch.no_grad():
            out_dim = self.model(self.X[0, :1]).shape[-1]
        self.binary = out_dim == 1

    def _unflat(self, flat):
        out, o = {}, 0
        for n, s in zip(self.names, self.shapes):
            k = int(np.prod(s))
            out[n] = flat[o:o + k].view(s)
            o += k
        return out

    def _loss(self, flat, x, y):
        out = functional_call(self.model, self._unflat(flat), (x.unsqueeze(0),))
        if self.binary:
            return torch.nn.functional.binary_cross_entropy(out.reshape(-1).clamp(1e-7, 1 - 1e-7),
                                                            y.float().reshape(-1))
        return torch.nn.functional.cross_entropy(out, y.long().reshape(-1))

    def _gather_rows(self, own):
        """[hi − lo, D] own rows → [N, D] all workers' rows (one all_gather, padded shards)."""
        buf = torch.zeros(self.per, own.shape[1], dtype=own.dtype, device=own.device)
        buf[:own.shape[0]] = own
        parts = comm.all_gather_flat(buf.reshape(-1))
        return torch.cat([q.view(self.per, -1) for q in parts])[:self.N]

    def _train_sharded(self):
        """The same iteration on this rank's workers lo:hi, gossip over all_gather."""
        loss_fn = vmap(self._loss)
        grad_fn = vmap(grad(self._loss))
        lo, hi = self.lo, self.hi
        mix_own = self.mix[lo:hi].contiguous()          # receiver rows of this rank
        x, z, om = self.x[lo:hi].clone(), self.z[lo:hi].clone(), self.omega[lo:hi].clone()
        per_iter = []
        for t in range(self.T * self.epoch):
            it = t % self.T
            xb, yb = self.X[lo:hi, it], self.Y[lo:hi, it]
            per_iter.append(loss_fn(z, xb, yb).double().sum())
            g = grad_fn(z, xb, yb)
            if self.wd:
                g = g + self.wd * z
            if self.mode == "LOCAL":
                z = z - self.lr * g
                x = z
                continue
            x = x - self.lr * g
            xa = self._gather_rows(x)
            x = ops.subset_aggregate(mix_own, xa) if xa.is_cuda else mix_own @ xa
            if self.mode == "PUSHSUM":
                om = mix_own @ self._gather_rows(om)
                z = x / om
            else:
                z = x
        losses = torch.stack(per_iter).to(torch.float64)
        comm.all_reduce_flat(losses)
        cum = torch.cumsum(losses, 0).cpu()
        self.regret_history = (cum / (self.N * torch.arange(1, len(per_iter) + 1))).tolist()
        self.z = self._gather_rows(z)
        return {"regret": self.regret_history, "params": self.z}

    def train(self):
        if self.world > 1:
            return self._train_sharded()
        loss_fn = vmap(self._loss)
        grad_fn = vmap(grad(self._loss))
        per_iter = []
        for t in range(self.T * self.epoch):
            it = t % self.T
            xb, yb = self.X[:, it], self.Y[:, it]
            losses = loss_fn(self.z, xb, yb)
            g = grad_fn(self.z, xb, yb)
            if self.wd:
                g = g + self.wd * self.z
            per_iter.append(losses.double().sum())
            if self.mode == "LOCAL":
                self.z = self.z - self.lr * g
                self.x = self.z
            else:
                self.x = self.x - self.lr * g
                self.x = ops.subset_aggregate(self.mix, self.x) if self.x.is_cuda else self.mix @ self.x
                if self.mode == "PUSHSUM":
                    self.omega = self.mix @ self.omega
                    self.z = self.x / self.omega
                else:
                    self.z = self.x
        cum = torch.cumsum(torch.stack(per_iter), 0).cpu()  # one host sync for the whole run
        self.regret_history = (cum / (self.N * torch.arange(1, len(per_iter) + 1))).tolist()
        logging.info("decentralized %s: final regret %.5f", self.mode, self.regret_history[-1])
        return {"regret": self.regret_history, "params": self.z}
