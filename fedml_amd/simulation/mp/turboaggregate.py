"""TurboAggregate-style secure FedAvg over message passing (reference:
`mpi_p2p_mp/turboaggregate/*`; the reference trains plain FedAvg and never calls its MPC
library — here the aggregation is actually secure, using ``core.mpc``).

Round protocol (server = rank 0, workers 1..W):
1. S2C_SYNC_MODEL: global model, client index, round.
2. worker trains, draws a fresh DH key pair and Shamir-shares its secret (threshold T) —
   C2S_PUBLIC_KEY carries ``pk`` and the per-peer shares (relayed by the server, which in a
   deployment would only see them encrypted to each peer).
3. S2C_PUBLIC_KEYS: every pk plus the shares addressed to that worker.
4. worker uploads C2S_MASKED_MODEL = Q(n_c/N · w_c) + pairwise masks (mod p), or C2S_DROPPED
   when it is scheduled to drop (``args.ta_dropout_ranks``; simulates a client that vanished
   after key exchange).
5. if anyone dropped: S2C_REVEAL → survivors return the shares they hold for the dropped
   workers (C2S_REVEAL_SHARES); the server reconstructs their secrets (BGW decoding) and
   strips their masks.
6. the server sums the masked uploads mod p (``fa_mod_sum`` HIP kernel on GPU), de-quantises and
   renormalises by the surviving sample mass → new global model.
"""
import logging
import time

import torch

from ...core.distributed import ClientManager, Message, ServerManager
from ...core.mpc import SecAggClient, SecureAggregator
from ...core.mpc.finite_field import DEFAULT_PRIME
from ...ops import mod_sum
from ...trainers import create_model_trainer
from .fl_protocol import FedAVGAggregator, FedAVGTrainer

MSG_S2C_SYNC_MODEL = 1
MSG_C2S_PUBLIC_KEY = 2
MSG_S2C_PUBLIC_KEYS = 3
MSG_C2S_MASKED_MODEL = 4
MSG_C2S_DROPPED = 5
MSG_S2C_REVEAL = 6
MSG_C2S_REVEAL_SHARES = 7
MSG_S2C_FINISH = 8


def _float_keys(sd):
    return [k for k, v in sd.items() if torch.is_floating_point(v)]


def flatten_float(sd):
    return torch.cat([sd[k].reshape(-1).double() for k in _float_keys(sd)])


def unflatten_float(flat, template):
    out, o = {}, 0
    for k, v in template.items():
        if torch.is_floating_point(v):
            n = v.numel()
            out[k] = flat[o:o + n].reshape(v.shape).to(v.dtype)
            o += n
        else:
            out[k] = v.clone()
    return out


class TAServerManager(ServerManager):
    def __init__(self, args, aggregator, comm, rank, size, backend, device):
        super().__init__(args, comm, rank, size, backend)
        self.agg = aggregator
        self.device = device
        self.round_idx = 0
        self.round_num = int(args.comm_round)
        self.W = size - 1
        self.T = int(getattr(args, "ta_threshold", max(1, self.W // 2)))
        self.frac_bits = int(getattr(args, "ta_frac_bits", 20))
        self.round_times = []
        self.dropped_history = []

    def register_message_receive_handlers(self):
        self.register_message_receive_handler(MSG_C2S_PUBLIC_KEY, self.handle_pk)
        self.register_message_receive_handler(MSG_C2S_MASKED_MODEL, self.handle_masked)
        self.register_message_receive_handler(MSG_C2S_DROPPED, self.handle_dropped)
        self.register_message_receive_handler(MSG_C2S_REVEAL_SHARES, self.handle_reveal)

    def start_round(self):
        self._t0 = time.time()
        self.clients = self.agg.client_sampling(self.round_idx, int(self.args.client_num_in_total), self.W)
        nums = [float(self.agg.train_data_local_num_dict[c]) for c in self.clients]
        self.n_of = {r: nums[r - 1] for r in range(1, self.size)}
        self.n_total = sum(nums)
        self.sa = SecureAggregator(self.W, self.T, DEFAULT_PRIME, self.frac_bits)
        self.shares_for = {r: {} for r in range(1, self.size)}
        self.masked, self.dropped, self.revealed = {}, set(), 0
        g = self.agg.get_global_model_params()
        for r in range(1, self.size):
            m = Message(MSG_S2C_SYNC_MODEL, 0, r)
            m.add_params("model_params", g)
            m.add_params("client_idx", int(self.clients[r - 1]))
            m.add_params("round_idx", self.round_idx)
            m.add_params("n_total", self.n_total)
            m.add_params("threshold", self.T)
            self.send_message(m)

    def handle_pk(self, msg):
        r = msg.get_sender_id()
        self.sa.add_public_key(r - 1, int(msg.get("pk")))
        for holder, share in enumerate(msg.get("shares")):
            self.shares_for[holder + 1][r - 1] = int(share)
        if len(self.sa.pks) < self.W:
            return
        for r2 in range(1, self.size):
            m = Message(MSG_S2C_PUBLIC_KEYS, 0, r2)
            m.add_params("pks", {str(k): v for k, v in self.sa.pks.items()})
            m.add_params("shares", {str(k): v for k, v in self.shares_for[r2].items()})
            self.send_message(m)

    def handle_masked(self, msg):
        self.masked[msg.get_sender_id() - 1] = msg.get("masked").to(self.device)
        self._maybe_unmask()

    def handle_dropped(self, msg):
        self.dropped.add(msg.get_sender_id() - 1)
        self._maybe_unmask()

    def _maybe_unmask(self):
        if len(self.masked) + len(self.dropped) < self.W:
            return
        if self.dropped:
            for c in self.masked:
                m = Message(MSG_S2C_REVEAL, 0, c + 1)
                m.add_params("dropped", sorted(self.dropped))
                self.send_message(m)
        else:
            self._finish_round()

    def handle_reveal(self, msg):
        holder = msg.get_sender_id() - 1
        for owner, share in msg.get("shares").items():
            self.sa.add_share(int(owner), holder, int(share))
        self.revealed += 1
        if self.revealed == len(self.masked):
            self._finish_round()

    def _finish_round(self):
        alive = sorted(self.masked)
        # fast path on device: Σ masked mod p in one kernel, then the aggregator strips dropout masks
        stacked = torch.stack([self.masked[c] for c in alive])
        summed = mod_sum(stacked, self.sa.p)
        avg = self.sa.unmask_sum(summed, alive)
        n_alive = sum(self.n_of[c + 1] for c in alive)
        avg = avg * (self.n_total / n_alive)
        g = self.agg.get_global_model_params()
        self.agg.set_global_model_params(unflatten_float(avg.cpu(), g))
        self.dropped_history.append(sorted(self.dropped))
        self.agg.test_on_server_for_all_clients(self.round_idx)
        self.round_times.append(time.time() - self._t0)
        self.round_idx += 1
        if self.round_idx >= self.round_num:
            for r in range(1, self.size):
                self.send_message(Message(MSG_S2C_FINISH, 0, r))
            self.finish()
            return
        self.start_round()


class TAClientManager(ClientManager):
    def __init__(self, args, trainer, comm, rank, size, backend, device):
        super().__init__(args, comm, rank, size, backend)
        self.trainer = trainer
        self.device = device
        self.W = size - 1
        self.frac_bits = int(getattr(args, "ta_frac_bits", 20))
        drop = getattr(args, "ta_dropout_ranks", None) or {}
        self.drop_rounds = {int(k): set(v) for k, v in drop.items()} if isinstance(drop, dict) else {}

    def register_message_receive_handlers(self):
        self.register_message_receive_handler(MSG_S2C_SYNC_MODEL, self.handle_sync)
        self.register_message_receive_handler(MSG_S2C_PUBLIC_KEYS, self.handle_pks)
        self.register_message_receive_handler(MSG_S2C_REVEAL, self.handle_reveal)
        self.register_message_receive_handler(MSG_S2C_FINISH, lambda m: self.finish())

    def handle_sync(self, msg):
        self.round_idx = int(msg.get("round_idx"))
        self.n_total = float(msg.get("n_total"))
        self.trainer.update_model(msg.get("model_params"))
        self.trainer.update_dataset(int(msg.get("client_idx")))
        weights, n = self.trainer.train(self.round_idx)
        self.template = weights
        self.x = flatten_float(weights).to(self.device) * (float(n) / self.n_total)
        self.sac = SecAggClient(self.rank - 1, self.W, int(msg.get("threshold")), DEFAULT_PRIME, self.frac_bits,
                                seed=hash((self.rank, self.round_idx, id(self))) & 0x7FFFFFFF)
        m = Message(MSG_C2S_PUBLIC_KEY, self.rank, 0)
        m.add_params("pk", self.sac.pk)
        m.add_params("shares", self.sac.sk_shares())
        self.send_message(m)

    def handle_pks(self, msg):
        self.held_shares = {int(k): int(v) for k, v in msg.get("shares").items()}
        if self.rank in self.drop_rounds.get(self.round_idx, ()):
            self.send_message(Message(MSG_C2S_DROPPED, self.rank, 0))
            return
        pks = {int(k): int(v) for k, v in msg.get("pks").items()}
        m = Message(MSG_C2S_MASKED_MODEL, self.rank, 0)
        m.add_params("masked", self.sac.masked_input(self.x, pks).cpu())
        self.send_message(m)

    def handle_reveal(self, msg):
        m = Message(MSG_C2S_REVEAL_SHARES, self.rank, 0)
        m.add_params("shares", {str(o): self.held_shares[o] for o in msg.get("dropped")})
        self.send_message(m)


def FedML_TurboAggregate_distributed(args, process_id, worker_number, comm, device, dataset, model,
                                     model_trainer=None, **_):
    (train_data_num, _, train_global, test_global, num_dict, train_local, test_local, _) = dataset[:8]
    backend = "LOOPBACK" if comm is not None else str(getattr(args, "backend", "TCP"))
    model_trainer = model_trainer or create_model_trainer(model, args)
    dev = device if device is not None else torch.device("cpu")
    if process_id == 0:
        agg = FedAVGAggregator(train_global, test_global, train_data_num, train_local, test_local, num_dict,
                               worker_number - 1, dev, args, model_trainer)
        s = TAServerManager(args, agg, comm, 0, worker_number, backend, dev)
        s.start_round()
        s.run()
        return {"global_model": agg.get_global_model_params(), "history": agg.history,
                "round_times": s.round_times, "dropped": s.dropped_history}
    tr = FedAVGTrainer(process_id - 1, train_local, num_dict, test_local, train_data_num, dev, args, model_trainer)
    c = TAClientManager(args, tr, comm, process_id, worker_number, backend, dev)
    c.run()
