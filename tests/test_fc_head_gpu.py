"""Fused classifier head (csrc/head_kernels.hip) against a plain PyTorch fp64 reference of the same op:
logits = P·Wᵀ + b from arena rows, softmax cross-entropy with per-row scales (1/batch, 0 for padding rows),
gW / gb accumulated into the gradient arena at the same offsets, dP = dl·W, per-client loss."""
import pytest
import torch

from fedml_amd.ops import nn_ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("C,N,F,K", [(3, 64, 256, 100), (2, 64, 512, 10), (5, 11, 64, 7), (1, 128, 256, 100)])
def test_fc_head_xent_matches_fp64(C, N, F, K):
    torch.manual_seed(0)
    P_ = 1000 + K * F + K + 3                      # odd arena stride: W rows are not 16-B aligned
    ow, ob = 17, 17 + K * F
    arena = torch.randn(C, P_, device=DEV) * 0.1
    garena = torch.randn(C, P_, device=DEV)
    g0 = garena.clone()
    pooled = torch.rand(C, N, F, device=DEV)
    labels = torch.randint(0, K, (C, N), device=DEV)
    rs = torch.full((C, N), 1.0 / N, device=DEV)
    rs[-1, N // 2:] = 0.0                          # padding rows of a ragged last client
    labels[-1, N // 2:] = -1
    dpool = torch.empty(C, N, F, device=DEV)
    loss_c = torch.empty(C, device=DEV)
    fits = (N * (F + 4) + N * K) * 4 <= 160 * 1024
    assert nn_ops.fc_head_xent(pooled, arena, ow, ob, labels, rs, garena, dpool, loss_c, C, N, F, K) == fits
    if not fits:      # too large for one workgroup's LDS: the caller keeps the library path, nothing written
        assert torch.equal(garena, g0)
        return
    torch.cuda.synchronize()
    for c in range(C):
        W = arena[c, ow:ow + K * F].view(K, F).double().requires_grad_(True)
        b = arena[c, ob:ob + K].double().requires_grad_(True)
        P = pooled[c].double().requires_grad_(True)
        z = P @ W.t() + b
        keep = rs[c] > 0
        lr = torch.nn.functional.cross_entropy(z[keep], labels[c][keep], reduction="none")
        loss = (lr * rs[c][keep].double()).sum()
        loss.backward()
        assert abs(float(loss_c[c]) - float(loss)) <= 1e-5 * abs(float(loss)) + 1e-6
        gW = (garena[c, ow:ow + K * F] - g0[c, ow:ow + K * F]).view(K, F).double()
        gb = (garena[c, ob:ob + K] - g0[c, ob:ob + K]).double()
        for got, ref in ((gW, W.grad), (gb, b.grad), (dpool[c].double(), P.grad)):
            assert float((got - ref).norm() / ref.norm()) < 1e-5
    untouched = torch.ones(P_, dtype=torch.bool)
    untouched[ow:ob + K] = False
    assert torch.equal(garena[:, untouched.to(DEV)], g0[:, untouched.to(DEV)])
