"""Error-feedback residuals of compressed client updates, sharded by owning rank.

A client's residual (the part of its update that quantisation / top-k dropped, fed back into its next
upload) lives only on the rank that trains that client. Every rank derives the same client→rank
assignment each round (reference RNG client sampling + the deterministic packer), so when a client
moves to another rank (partial participation) its row is handed over point-to-point before local
training; with full participation (the north-star configs) clients never move and each rank holds
only ~K/world rows. Checkpoints gather the dense [K, P] matrix (rows are disjoint across ranks, so one
sum all-reduce assembles it).
"""
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ...parallel import comm


class ShardedResiduals:
    def __init__(self, P: int, device, rank: int = 0, world: int = 1):
        self.P = int(P)
        self.device = torch.device(device)
        self.rank, self.world = rank, world
        self.rows: Dict[int, torch.Tensor] = {}
        self.owner: Dict[int, int] = {}

    def __getitem__(self, cid: int) -> torch.Tensor:
        """This rank's row of client ``cid`` (zeros on first use). Ownership is never changed here: only
        ``migrate`` (the same call on every rank) assigns owners, so all ranks keep the same owner map."""
        cid = int(cid)
        if cid < 0:
            raise KeyError(f"client id {cid}: padding slots have no residual row")
        row = self.rows.get(cid)
        if row is None:
            row = self.rows[cid] = torch.zeros(self.P, dtype=torch.float32, device=self.device)
        return row

    def nbytes(self) -> int:
        return sum(r.numel() * 4 for r in self.rows.values())

    def migrate(self, assignment: Dict[int, int]):
        """Move the rows of clients whose training rank changes this round (identical call on every
        rank; clients are visited in sorted order so sends and receives pair up)."""
        reqs: List = []
        for cid in sorted(assignment):
            new = assignment[cid]
            old = self.owner.get(cid)
            if old is None or old == new:
                self.owner[cid] = new
                continue
            if self.rank == old:
                row = self.rows.pop(cid)
                reqs.append((dist.isend(row, dst=new), row))      # keep the buffer alive until done
            elif self.rank == new:
                buf = torch.empty(self.P, dtype=torch.float32, device=self.device)
                self.rows[cid] = buf
                reqs.append((dist.irecv(buf, src=old), buf))
            self.owner[cid] = new
        for r, _ in reqs:
            r.wait()

    def dense(self, K: int) -> torch.Tensor:
        """[K, P] with every client's row (all ranks must call; rows are disjoint → sum all-reduce)."""
        out = torch.zeros(K, self.P, dtype=torch.float32, device=self.device)
        for cid, row in self.rows.items():
            out[cid].copy_(row)
        if comm.is_dist():
            comm.all_reduce_flat(out.view(-1))
        return out

    def load_dense(self, dense: torch.Tensor, owners: Optional[Dict[int, int]] = None):
        """Restore from a dense [K, P] matrix: rows go to their owner (default: this rank keeps all)."""
        self.rows.clear()
        self.owner.clear()
        for cid in range(dense.shape[0]):
            o = self.rank if owners is None else owners.get(cid, self.rank)
            self.owner[cid] = o
            if o == self.rank and bool(dense[cid].abs().max() > 0):
                self.rows[cid] = dense[cid].to(self.device, torch.float32).clone()
