"""Finite-field MPC primitives (reference: `turboaggregate/mpc_function.py:4-281`).

Same API surface — modular inverse, Lagrange coefficients, BGW (Shamir) encode/decode, LCC
encode/decode (with/without explicit randomness and evaluation points), additive secret
sharing, Diffie–Hellman key generation/agreement — with two differences:

* every modular product/accumulation is exact: ``mod_matmul`` reduces after each multiply, so
  any prime ``p < 2**31`` is safe (the reference's ``np.dot`` of int64 residues silently
  overflows once ``K·p² > 2**63``);
* large encodes (``[K+T] × d`` with d = model size) run on the GPU through the
  ``fa_mod_matmul`` HIP kernel when the operand is a CUDA tensor.

Arrays are int64 numpy (or torch int64) residues in ``[0, p)``.
"""
import numpy as np
import torch

DEFAULT_PRIME = 2 ** 31 - 1  # Mersenne prime: products of residues fit in int64


def modular_inv(a, p):
    a = int(a) % int(p)
    if a == 0:
        raise ZeroDivisionError("0 has no inverse mod p")
    return pow(a, -1, int(p))


def divmod(_num, _den, _p):  # noqa: A001 - reference name
    return (int(_num) % _p) * modular_inv(_den, _p) % _p


def PI(vals, p):
    acc = 1
    for v in vals:
        acc = acc * (int(v) % p) % p
    return acc


def gen_Lagrange_coeffs(alpha_s, beta_s, p, is_K1=0):
    """U[i, j] = ∏_{o≠β_j} (α_i − o) / (β_j − o)  — evaluates at α the interpolant through β."""
    alphas = list(alpha_s)[:1] if is_K1 == 1 else list(alpha_s)
    betas = [int(b) for b in beta_s]
    U = np.zeros((len(alphas), len(betas)), dtype=np.int64)
    for j, bj in enumerate(betas):
        den = PI([bj - o for o in betas if o != bj], p)
        inv = modular_inv(den, p)
        for i, ai in enumerate(alphas):
            U[i, j] = PI([int(ai) - o for o in betas if o != bj], p) * inv % p
    return U


def mod_matmul(A, B, p):
    """(A @ B) mod p for int64 residues, exact. A: [M,K], B: [K, ...]."""
    if isinstance(B, torch.Tensor):
        from ...ops import mod_matmul as dev_mm
        At = A if isinstance(A, torch.Tensor) else torch.as_tensor(np.asarray(A, dtype=np.int64))
        return dev_mm(At.to(B.device), B, int(p))
    A = np.asarray(A, dtype=np.int64) % p
    B = np.asarray(B, dtype=np.int64) % p
    shp = B.shape[1:]
    B2 = B.reshape(B.shape[0], -1)
    out = np.zeros((A.shape[0], B2.shape[1]), dtype=np.int64)
    for k in range(A.shape[1]):
        out = (out + (A[:, k:k + 1] * B2[k:k + 1, :]) % p) % p
    return out.reshape((A.shape[0],) + shp)


def _rand(shape, p, rng=None):
    rng = rng if rng is not None else np.random
    return rng.randint(0, p, size=shape).astype(np.int64) if hasattr(rng, "randint") else \
        rng.integers(0, p, size=shape, dtype=np.int64)


def BGW_encoding(X, N, T, p, rng=None):
    """Shamir shares: share_i = Σ_t R_t α_i^t with R_0 = X, α_i = i (1-based). → [N, m, d]."""
    X = np.asarray(X, dtype=np.int64)
    R = np.concatenate([X[None] % p, _rand((T,) + X.shape, p, rng)], 0)
    V = np.array([[pow(i, t, p) for t in range(T + 1)] for i in range(1, N + 1)], dtype=np.int64)
    return mod_matmul(V, R, p)


def gen_BGW_lambda_s(alpha_s, p):
    return gen_Lagrange_coeffs([0], alpha_s, p)


def BGW_decoding(f_eval, worker_idx, p):
    """Reconstruct f(0) from the shares of workers ``worker_idx`` (0-based; α = idx+1)."""
    alphas = [int(i) + 1 for i in worker_idx]
    lam = gen_BGW_lambda_s(alphas, p)
    return mod_matmul(lam, np.asarray(f_eval, dtype=np.int64), p)


def _lcc_points(N, K, T, p):
    n_beta = K + T
    sb, sa = -(n_beta // 2), -(N // 2)
    beta_s = [(b % p) for b in range(sb, sb + n_beta)]
    alpha_s = [(a % p) for a in range(sa, sa + N)]
    return alpha_s, beta_s


def LCC_encoding_w_Random(X, R_, N, K, T, p):
    X = np.asarray(X, dtype=np.int64)
    m = X.shape[0]
    sub = np.concatenate([X[:(m // K) * K].reshape((K, m // K) + X.shape[1:]),
                          np.asarray(R_, dtype=np.int64).reshape((T, m // K) + X.shape[1:])], 0)
    alpha_s, beta_s = _lcc_points(N, K, T, p)
    return mod_matmul(gen_Lagrange_coeffs(alpha_s, beta_s, p), sub, p)


def LCC_encoding(X, N, K, T, p, rng=None):
    X = np.asarray(X, dtype=np.int64)
    R = _rand((T, X.shape[0] // K) + X.shape[1:], p, rng)
    return LCC_encoding_w_Random(X, R, N, K, T, p)


def LCC_encoding_w_Random_partial(X, R_, N, K, T, p, worker_idx):
    full = LCC_encoding_w_Random(X, R_, N, K, T, p)
    return full[np.asarray(worker_idx)]


def LCC_decoding(f_eval, f_deg, N, K, T, worker_idx, p):
    """Recover the K data blocks from ``(K+T-1)·f_deg + 1`` evaluations at workers ``worker_idx``.
    Decodes at the same β points the encoder used (the reference re-derives β from K alone,
    which only coincides with the encoder's points when T = 0)."""
    alpha_s, beta_s = _lcc_points(N, K, T, p)
    need = (K + T - 1) * f_deg + 1
    idx = list(worker_idx)[:need]
    alpha_eval = [alpha_s[i] for i in idx]
    U = gen_Lagrange_coeffs(beta_s[:K], alpha_eval, p)
    return mod_matmul(U, np.asarray(f_eval, dtype=np.int64)[:len(idx)], p)


def Gen_Additive_SS(d, n_out, p, rng=None):
    """``[n_out, d]`` additive shares of ZERO: each column sums to 0 mod p (reference semantics)."""
    head = _rand((n_out - 1, d), p, rng)
    last = (-(head.sum(0) % p)) % p
    return np.concatenate([head, last[None]], 0)


def additive_share(X, n, p, rng=None):
    """Split X into n additive shares (Σ shares ≡ X mod p)."""
    X = np.asarray(X, dtype=np.int64) % p
    s = _rand((n - 1,) + X.shape, p, rng)
    last = (X - s.sum(0) % p) % p
    return np.concatenate([s, last[None]], 0)


def LCC_encoding_with_points(X, alpha_s, beta_s, p):
    """Rows of X sit at points ``alpha_s``; evaluate their interpolant at ``beta_s``."""
    X = np.asarray(X, dtype=np.int64)
    U = gen_Lagrange_coeffs(beta_s, alpha_s, p)
    return mod_matmul(U, X, p)


def LCC_decoding_with_points(f_eval, eval_points, target_points, p):
    U = gen_Lagrange_coeffs(target_points, eval_points, p)
    return mod_matmul(U, f_eval, p)


def my_pk_gen(my_sk, p, g):
    """Diffie–Hellman public key g^sk mod p (``g == 0`` → identity, as in the reference)."""
    return int(my_sk) % int(p) if g == 0 else pow(int(g), int(my_sk), int(p))


def my_key_agreement(my_sk, u_pk, p, g):
    return int(my_sk) * int(u_pk) % int(p) if g == 0 else pow(int(u_pk), int(my_sk), int(p))


# ---- fixed-point embedding of real tensors --------------------------------------------------
def quantize_to_field(x: torch.Tensor, p=DEFAULT_PRIME, frac_bits=20) -> torch.Tensor:
    """round(x·2^frac_bits) mapped to [0,p) (negatives wrap). Exact for |x|·2^frac_bits < p/2."""
    q = torch.round(x.double() * (1 << frac_bits)).to(torch.int64)
    return torch.remainder(q, p)


def dequantize_from_field(q: torch.Tensor, p=DEFAULT_PRIME, frac_bits=20) -> torch.Tensor:
    q = torch.remainder(q.to(torch.int64), p)
    signed = torch.where(q > p // 2, q - p, q)
    return signed.double() / (1 << frac_bits)
