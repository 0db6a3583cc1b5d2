"""Client data containers.

The reference hands trainers either pre-batched python lists of ``(x, y)``
tensors (`data/MNIST/data_loader.py:75-98`) or torch ``DataLoader`` objects
(`data/cifar10/data_loader.py:312-374`). ``ClientData`` offers both behaviours
(iteration yields batches, ``len`` = number of batches, indexing) while keeping
the client's samples as two contiguous tensors, which is what the batched
virtual-client engine consumes directly (``.x``, ``.y``) — possibly already
resident in HBM (``.to(device)``).
"""
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch


class ClientData:
    def __init__(self, x: torch.Tensor, y: torch.Tensor, batch_size: int, shuffle: bool = False,
                 seed: Optional[int] = None, drop_last: bool = False, transform=None):
        assert len(x) == len(y)
        self.x = x
        self.y = y
        self.batch_size = int(batch_size) if batch_size and batch_size > 0 else max(1, len(x))
        self.shuffle = shuffle
        self.seed = seed
        self.drop_last = drop_last
        self.transform = transform
        self._epoch = 0

    # ---- python-list / DataLoader behaviour -------------------------------------
    @property
    def num_samples(self) -> int:
        return len(self.x)

    @property
    def dataset(self):
        return self

    def __len__(self) -> int:
        n = len(self.x)
        if self.drop_last:
            return n // self.batch_size
        return (n + self.batch_size - 1) // self.batch_size

    def _order(self):
        n = len(self.x)
        if not self.shuffle:
            return None
        g = torch.Generator()
        g.manual_seed((self.seed or 0) * 1000003 + self._epoch)
        self._epoch += 1
        return torch.randperm(n, generator=g)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        order = self._order()
        nb = len(self)
        for b in range(nb):
            s = slice(b * self.batch_size, min((b + 1) * self.batch_size, len(self.x)))
            if order is None:
                xb, yb = self.x[s], self.y[s]
            else:
                idx = order[s]
                xb, yb = self.x[idx], self.y[idx]
            if self.transform is not None:
                xb = self.transform(xb)
            yield xb, yb

    def __getitem__(self, i):
        if i < 0:
            i += len(self)
        s = slice(i * self.batch_size, min((i + 1) * self.batch_size, len(self.x)))
        return self.x[s], self.y[s]

    def to(self, device):
        return ClientData(self.x.to(device), self.y.to(device), self.batch_size, self.shuffle, self.seed,
                          self.drop_last, self.transform)

    def with_batch_size(self, bs):
        return ClientData(self.x, self.y, bs, self.shuffle, self.seed, self.drop_last, self.transform)

    def __repr__(self):
        return f"ClientData(n={len(self.x)}, batch_size={self.batch_size}, x={tuple(self.x.shape)})"


def concat_client_data(parts: Sequence[ClientData], batch_size: Optional[int] = None) -> ClientData:
    parts = [p for p in parts if p is not None and p.num_samples > 0]
    if not parts:
        return ClientData(torch.zeros(0), torch.zeros(0, dtype=torch.long), 1)
    x = torch.cat([p.x for p in parts])
    y = torch.cat([p.y for p in parts])
    return ClientData(x, y, batch_size or parts[0].batch_size)


def batches_to_client_data(batches: List[Tuple[torch.Tensor, torch.Tensor]], batch_size: int) -> ClientData:
    """Adapt a reference-style list of (x, y) batches."""
    if isinstance(batches, ClientData):
        return batches
    xs = [b[0] for b in batches]
    ys = [b[1] for b in batches]
    return ClientData(torch.cat(xs) if xs else torch.zeros(0), torch.cat(ys) if ys else torch.zeros(0), batch_size)


def split_client_data(cd: ClientData, n_parts: int) -> List[ClientData]:
    """Shard one client's samples across ``n_parts`` data-parallel ranks
    (reference: `data/data_loader_cross_silo.py:9-47`; pads by wrapping so every shard has equal size,
    the DistributedSampler convention)."""
    n = cd.num_samples
    per = (n + n_parts - 1) // n_parts
    idx = np.arange(per * n_parts) % max(n, 1)
    out = []
    for r in range(n_parts):
        sel = torch.as_tensor(idx[r::n_parts])
        out.append(ClientData(cd.x[sel], cd.y[sel], cd.batch_size, cd.shuffle, cd.seed))
    return out
