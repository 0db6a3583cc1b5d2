"""Device-resident client data store.

All training samples of the federation live in HBM as one tensor ``x_all [N, ...]``
(``y_all [N, ...]``) — CIFAR-100 is 614 MB fp32, trivial next to 288 GB — plus a
per-client index table. Each round a GPU gathers mini-batches for *its*
virtual clients straight from that tensor: no host→device copy per batch and
no per-client DataLoader (reference hot loop 3).
"""
from typing import Dict, List, Optional

import torch


def _fmix32(x: torch.Tensor) -> torch.Tensor:
    """murmur3 finaliser on int64 tensors holding 32-bit values (products stay below 2^63)."""
    m = 0xFFFFFFFF
    x = x & m
    x = x ^ (x >> 16)
    x = (x * 0x85EBCA6B) & m
    x = x ^ (x >> 13)
    x = (x * 0xC2B2AE35) & m
    return x ^ (x >> 16)


def hash_uniform(key: int, a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Deterministic uniform [0, 1) keys from (key, a, b) integer tensors (broadcast): a counter-based
    hash, so a client's draws do not depend on a generator's position."""
    h = _fmix32(a.to(torch.int64) * 0x9E3779B1 + (key & 0xFFFFFFFF))
    h = _fmix32(h + b.to(torch.int64) * 0x7FEB352D)
    return h.to(torch.float32) * (1.0 / 4294967296.0)


class DeviceClientStore:
    def __init__(self, x_all: torch.Tensor, y_all: torch.Tensor, client_offsets: List[int], client_counts: List[int]):
        self.x_all = x_all
        self.y_all = y_all
        self.offsets = torch.as_tensor(client_offsets, dtype=torch.int64, device=x_all.device)
        self.counts = torch.as_tensor(client_counts, dtype=torch.int64, device=x_all.device)
        self.counts_host = list(int(c) for c in client_counts)
        self.device = x_all.device

    @property
    def num_clients(self):
        return len(self.counts_host)

    @classmethod
    def from_client_data(cls, train_local: Dict[int, "ClientData"], device, dtype=None) -> "DeviceClientStore":
        ids = sorted(train_local)
        xs, ys, offs, cnts = [], [], [], []
        off = 0
        for cid in ids:
            cd = train_local[cid]
            if hasattr(cd, "x"):
                cx, cy = cd.x, cd.y
            else:   # a user's loader (DataLoader / list of (x, y) batches): one pass to stage it in HBM
                batches = list(cd)
                cx = torch.cat([torch.as_tensor(b[0]) for b in batches])
                cy = torch.cat([torch.as_tensor(b[1]) for b in batches])
            xs.append(cx)
            ys.append(cy)
            offs.append(off)
            cnts.append(len(cx))
            off += len(cx)
        x = torch.cat(xs).to(device)
        if dtype is not None and x.is_floating_point():
            x = x.to(dtype)
        y = torch.cat(ys).to(device)
        return cls(x, y, offs, cnts)

    @classmethod
    def synthetic_on_device(cls, spec, counts: List[int], device, seed: int = 0, dtype=torch.float32,
                            num_classes: Optional[int] = None) -> "DeviceClientStore":
        """Generate a class-conditional synthetic dataset directly in HBM (bench path; same
        distribution family as ``data.synthetic`` but drawn with the device RNG)."""
        from ...data.synthetic import SyntheticGenerator
        gen = SyntheticGenerator(spec, seed=seed)
        n = int(sum(counts))
        g = torch.Generator(device=device)
        g.manual_seed(seed + 99)
        k = num_classes or spec.num_classes
        y = torch.randint(0, k, (n,), generator=g, device=device)
        if spec.kind == "image":
            proto = gen.proto.to(device)
            x = torch.empty((n,) + tuple(spec.shape), dtype=dtype, device=device)
            chunk = 8192
            for s in range(0, n, chunk):
                e = min(n, s + chunk)
                noise = torch.randn((e - s,) + tuple(spec.shape), generator=g, device=device)
                x[s:e] = (0.5 * proto[y[s:e]] + 0.5 * noise).to(dtype)
        elif spec.kind == "vector":
            proto = gen.proto.to(device)
            x = (proto[y] + torch.randn((n,) + tuple(spec.shape), generator=g, device=device)).to(dtype)
        else:
            probs = gen.token_probs.to(device)
            x = torch.multinomial(probs[y], spec.shape[0], replacement=True, generator=g)
        offs, off = [], 0
        for c in counts:
            offs.append(off)
            off += int(c)
        return cls(x, y, offs, counts)

    # ------------------------------------------------------------------------------------------
    def epoch_order(self, slots: torch.Tensor, n_max: int, generator: Optional[torch.Generator] = None,
                    shuffle: bool = True, key: Optional[int] = None) -> torch.Tensor:
        """Global sample indices [C, n_max] for the given client slots (−1 for padding).

        ``key`` (int): shuffle by a counter hash of (key, client id, position) instead of ``generator``
        — every client's order is then a function of (seed, round, epoch, client) only, independent of
        which rank / slot trains it (world-size-invariant runs, exact resume from the round index)."""
        C = len(slots)
        counts = self.counts[slots]                           # [C]
        ar = torch.arange(n_max, device=self.device).unsqueeze(0).expand(C, n_max)
        valid = ar < counts.unsqueeze(1)
        if shuffle and key is not None:
            keys = hash_uniform(int(key), slots.to(self.device).view(C, 1), ar)
            keys = torch.where(valid, keys, torch.full_like(keys, 2.0))
            local = torch.argsort(keys, dim=1)
        elif shuffle:
            keys = torch.rand(C, n_max, generator=generator, device=self.device)
            keys = torch.where(valid, keys, torch.full_like(keys, 2.0))
            local = torch.argsort(keys, dim=1)
        else:
            local = ar
        idx = self.offsets[slots].unsqueeze(1) + local
        return torch.where(valid, idx, torch.full_like(idx, -1))

    def gather(self, idx: torch.Tensor):
        """idx [C, b] (−1 = padding) → x [C, b, ...], y [C, b, ...], mask [C, b]."""
        mask = idx >= 0
        safe = idx.clamp_min(0)
        return self.x_all[safe], self.y_all[safe], mask
