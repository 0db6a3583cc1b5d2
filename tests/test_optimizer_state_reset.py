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


def _check_inactive(dev):
    """A client idle in a step (active 0, step counter still at 1) keeps every piece of its state — the HIP
    kernel skips its row entirely; the CPU fallback must not reset its moments or decay its weights."""
    torch.manual_seed(1)
    C, P = 3, 517
    for amsgrad in (False, True):
        p = torch.randn(C, P, device=dev)
        m1, m2 = torch.randn(C, P, device=dev), torch.rand(C, P, device=dev)
        vm = torch.rand(C, P, device=dev) if amsgrad else None
        sh = p.to(torch.bfloat16)
        before = [t.clone() for t in (p, m1, m2) + ((vm,) if amsgrad else ())] + [sh.clone()]
        act = torch.tensor([1.0, 0.0, 1.0], device=dev)
        ops.adam_step(p, torch.randn(C, P, device=dev), m1, m2, torch.ones(C, device=dev), 1e-2, weight_decay=0.1,
                      amsgrad=amsgrad, max_exp_avg_sq=vm, decoupled=True, active=act, shadow=sh)
        after = [p, m1, m2] + ([vm] if amsgrad else []) + [sh]
        for a, b in zip(before, after):
            assert torch.equal(a[1], b[1])          # idle client: untouched
            assert not torch.equal(a[0], b[0])      # active client: updated


def test_adam_inactive_client_keeps_state_cpu():
    _check_inactive("cpu")


@pytest.mark.gpu
def test_adam_inactive_client_keeps_state_gpu():
    _check_inactive("cuda")


def test_broadcast_rows_cpu():
    dst = torch.randn(4, 10)
    src = torch.randn(10)
    ops.broadcast_rows_(dst, src)
    assert torch.equal(dst, src.expand(4, 10))


@pytest.mark.gpu
def test_adam_first_step_ignores_stale_moments_gpu():
    _check_fresh("cuda")


@pytest.mark.gpu
@pytest.mark.parametrize("C,P,ld", [(3, 1001, 1001), (5, 4096, 4100), (2, 7, 9), (19, 5000, 5004), (17, 333, 333)])
def test_broadcast_rows_gpu(C, P, ld):
    buf = torch.randn(C, ld, device="cuda")
    dst = buf[:, :P]
    src = torch.randn(P, device="cuda")
    keep = buf[:, P:].clone()
    ops.broadcast_rows_(dst, src)
    torch.cuda.synchronize()
    assert torch.equal(dst, src.expand(C, P))
    assert torch.equal(buf[:, P:], keep)   # the padding columns past P are untouched
