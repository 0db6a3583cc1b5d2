"""Per-round optimizer-state resets without fill passes: Adam's first step (t = 1) starts from zero moments
whatever the moment buffers hold (the engine no longer zeroes m1/m2/vmax between rounds), and the global
model reaches every client row through one broadcast launch (``ops.broadcast_rows_``)."""
import pytest
import torch

from fedml_amd import ops


def _adam(dev, m_fill, amsgrad):
    torch.manual_seed(0)
    C, P = 3, 1031
    p = torch.randn(C, P, device=dev)
    g = torch.randn(C, P, device=dev)
    m1 = torch.full((C, P), m_fill, device=dev)
    m2 = torch.full((C, P), m_fill, device=dev)
    vm = torch.full((C, P), m_fill, device=dev) if amsgrad else None
    step = torch.tensor([1.0, 1.0, 1.0], device=dev)
    ops.adam_step(p, g, m1, m2, step, 1e-2, weight_decay=0.01, amsgrad=amsgrad, max_exp_avg_sq=vm, decoupled=True)
    return p, m1, m2


def _check_fresh(dev):
    for amsgrad in (False, True):
        ref = _adam(dev, 0.0, amsgrad)
        for fill in (3.0, float("nan")):
            got = _adam(dev, fill, amsgrad)
            for a, b in zip(ref, got):
                assert torch.equal(a, b)


def test_adam_first_step_ignores_stale_moments_cpu():
    _check_fresh("cpu")


def test_broadcast_rows_cpu():
    dst = torch.randn(4, 10)
    src = torch.randn(10)
    ops.broadcast_rows_(dst, src)
    assert torch.equal(dst, src.expand(4, 10))


@pytest.mark.gpu
def test_adam_first_step_ignores_stale_moments_gpu():
    _check_fresh("cuda")


@pytest.mark.gpu
@pytest.mark.parametrize("C,P,ld", [(3, 1001, 1001), (5, 4096, 4100), (2, 7, 9)])
def test_broadcast_rows_gpu(C, P, ld):
    buf = torch.randn(C, ld, device="cuda")
    dst = buf[:, :P]
    src = torch.randn(P, device="cuda")
    keep = buf[:, P:].clone()
    ops.broadcast_rows_(dst, src)
    torch.cuda.synchronize()
    assert torch.equal(dst, src.expand(C, P))
    assert torch.equal(buf[:, P:], keep)   # the padding columns past P are untouched
