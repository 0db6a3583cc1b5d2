"""Dropout-resilient secure aggregation built on the finite-field library — what TurboAggregate
uses it for (the reference ships `mpc_function.py` but never calls it).

Protocol (pairwise-mask SecAgg, Bonawitz et al. 2017, single-mask variant):
1. every client draws a DH secret ``sk_i`` and publishes ``pk_i = g^sk_i mod q``;
2. each client Shamir-shares ``sk_i`` (``BGW_encoding``, threshold T) to its peers;
3. client i uploads ``y_i = Q(x_i) + Σ_{j>i} PRG(s_ij) − Σ_{j<i} PRG(s_ij)  (mod p)`` with
   ``s_ij = pk_j^sk_i`` — the masks cancel in the sum;
4. for each client that dropped after step 2, the server gathers T+1 shares of its ``sk``
   (``BGW_decoding``), recomputes its pairwise masks with the survivors and removes them.

Vectors are int64 residues on the compute device; the PRG is a counter-based SplitMix64 in
torch int64 ops, so CPU and GPU parties derive identical masks. Simplifications versus the
paper (documented, not hidden): no self-mask b_i (a dropped-then-late client could be
unmasked), and share delivery is not encrypted — a transport-level concern here.
"""
import random
from typing import Dict, List

import numpy as np
import torch

from .finite_field import (DEFAULT_PRIME, BGW_decoding, BGW_encoding, dequantize_from_field, my_key_agreement,
                           my_pk_gen, quantize_to_field)

DH_GENERATOR = 7  # primitive root mod 2^31-1


def _u64(c):
    return c - (1 << 64) if c >= (1 << 63) else c


_C1, _C2, _C3 = _u64(0x9E3779B97F4A7C15), _u64(0xBF58476D1CE4E5B9), _u64(0x94D049BB133111EB)


def _lsr(z, k):
    return (z >> k) & ((1 << (64 - k)) - 1)


def prg(seed: int, d: int, p: int = DEFAULT_PRIME, device="cpu") -> torch.Tensor:
    z = torch.arange(d, dtype=torch.int64, device=device) + _u64((int(seed) * 0x9E3779B97F4A7C15) % (1 << 64))
    z = z * _C1
    z = (z ^ _lsr(z, 30)) * _C2
    z = (z ^ _lsr(z, 27)) * _C3
    z = z ^ _lsr(z, 31)
    return _lsr(z, 33) % p


def pairwise_mask(i: int, sk_i: int, pks: Dict[int, int], d: int, p=DEFAULT_PRIME, device="cpu", peers=None):
    m = torch.zeros(d, dtype=torch.int64, device=device)
    for j in (peers if peers is not None else pks):
        if j == i:
            continue
        s = my_key_agreement(sk_i, pks[j], DEFAULT_PRIME, DH_GENERATOR)
        r = prg(s, d, p, device)
        m = (m + r) % p if j > i else (m - r) % p
    return m


class SecAggClient:
    def __init__(self, cid: int, n: int, threshold: int, p=DEFAULT_PRIME, frac_bits=20, seed=None):
        self.cid, self.n, self.T, self.p, self.frac_bits = cid, n, threshold, p, frac_bits
        rng = random.Random(seed)
        self.sk = rng.randrange(2, DEFAULT_PRIME - 1)
        self.pk = my_pk_gen(self.sk, DEFAULT_PRIME, DH_GENERATOR)
        self._np_rng = np.random.RandomState(rng.randrange(1 << 31))

    def sk_shares(self) -> List[int]:
        """Shamir shares of sk for clients 0..n-1 (client j gets share j; α_j = j+1)."""
        sh = BGW_encoding(np.array([[self.sk]], dtype=np.int64), self.n, self.T, DEFAULT_PRIME, rng=self._np_rng)
        return [int(sh[j, 0, 0]) for j in range(self.n)]

    def masked_input(self, x: torch.Tensor, pks: Dict[int, int]) -> torch.Tensor:
        q = quantize_to_field(x.reshape(-1), self.p, self.frac_bits).to(x.device)
        return (q + pairwise_mask(self.cid, self.sk, pks, q.numel(), self.p, x.device)) % self.p


class SecureAggregator:
    def __init__(self, n: int, threshold: int, p=DEFAULT_PRIME, frac_bits=20):
        self.n, self.T, self.p, self.frac_bits = n, threshold, p, frac_bits
        self.pks: Dict[int, int] = {}
        self.shares: Dict[int, Dict[int, int]] = {}  # owner -> {holder: share}

    def add_public_key(self, cid, pk):
        self.pks[cid] = int(pk)

    def add_share(self, owner, holder, share):
        self.shares.setdefault(owner, {})[holder] = int(share)

    def recover_sk(self, owner: int, holders: List[int]) -> int:
        hs = [h for h in holders if h in self.shares.get(owner, {})][: self.T + 1]
        if len(hs) < self.T + 1:
            raise RuntimeError(f"cannot recover client {owner}: {len(hs)} shares < T+1={self.T + 1}")
        f = np.array([[[self.shares[owner][h]]] for h in hs], dtype=np.int64)
        return int(BGW_decoding(f.reshape(len(hs), 1), hs, DEFAULT_PRIME)[0, 0])

    def aggregate(self, masked: Dict[int, torch.Tensor]) -> torch.Tensor:
        """Σ over survivors of the de-masked fixed-point inputs, as float64."""
        from ...ops import mod_sum
        alive = sorted(masked)
        return self.unmask_sum(mod_sum(torch.stack([masked[c] for c in alive]), self.p), alive)

    def unmask_sum(self, summed: torch.Tensor, alive: List[int]) -> torch.Tensor:
        """Strip the pairwise masks dropped clients left in the survivors' uploads."""
        acc = summed
        for k in [c for c in self.pks if c not in alive]:
            sk_k = self.recover_sk(k, alive)
            # survivor j's upload holds +PRG(s_jk) if k>j, −PRG(s_jk) if k<j (s_jk = s_kj):
            # pairwise_mask(k, …) over the survivors is exactly the negation of that residue.
            acc = (acc + pairwise_mask(k, sk_k, self.pks, acc.numel(), self.p, acc.device, peers=alive)) % self.p
        return dequantize_from_field(acc, self.p, self.frac_bits)
