"""GroupNorm HIP kernels (``csrc/gn_kernels.hip``) vs the fp32 PyTorch reference: forward, dx, dγ, dβ,
single-model and client-stacked (per-client affine read from strided arena views), fused ReLU."""
import pytest
import torch

from fedml_amd import ops
from fedml_amd.ops.norm_ops import FusedGroupNorm, _gn_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, tol):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    ref = b.abs().max().item() + 1e-6
    assert err <= tol * ref, f"max err {err} vs ref scale {ref}"


@pytest.mark.parametrize("N,ch,groups,clients,hw,dtype,relu,affine", [
    (4, 64, 2, 1, (8, 8), torch.float32, False, True),
    (3, 32, 4, 3, (5, 7), torch.float32, True, True),
    (8, 128, 4, 2, (16, 16), torch.bfloat16, False, True),
    (2, 512, 16, 1, (4, 4), torch.bfloat16, True, False),
    (2, 64, 2, 1, (56, 56), torch.float32, False, True),
])
def test_group_norm_fwd_bwd(N, ch, groups, clients, hw, dtype, relu, affine):
    torch.manual_seed(0)
    x = (torch.randn(N, clients * ch, *hw) * 2 + 0.3).to(dtype)
    if affine:
        # per-client affine as strided rows of a wider fp32 "arena" (client stride > ch)
        arena = torch.randn(clients, 3 * ch + 5)
        w0 = (1 + 0.1 * arena[:, :ch]).contiguous()
        b0 = (0.1 * arena[:, ch:2 * ch]).contiguous()
        big = torch.zeros(clients, 3 * ch + 5, device=DEV)
        big[:, 5:5 + ch] = w0.to(DEV)
        big[:, 5 + ch:5 + 2 * ch] = b0.to(DEV)
        wv = big[:, 5:5 + ch].detach().requires_grad_(True)
        bv = big[:, 5 + ch:5 + 2 * ch].detach().requires_grad_(True)
        if clients == 1:
            wv = wv.detach().reshape(ch).requires_grad_(True)
            bv = bv.detach().reshape(ch).requires_grad_(True)
    else:
        w0 = b0 = wv = bv = None
    xg = x.to(DEV).requires_grad_(True)
    y = ops.group_norm(xg, groups, wv, bv, 1e-5, relu=relu, clients=clients)
    gy = torch.randn(y.shape).to(dtype)
    y.backward(gy.to(DEV))
    # reference on the same (rounded) inputs in fp32
    xr = x.float().requires_grad_(True)
    wr = w0.clone().requires_grad_(True) if affine else None
    br = b0.clone().requires_grad_(True) if affine else None
    yr = _gn_ref(xr, groups, wr, br, 1e-5, relu, clients)
    yr.backward(gy.float())
    tol = 2e-2 if dtype == torch.bfloat16 else 2e-4
    _close(y, yr, tol)
    _close(xg.grad, xr.grad, 3 * tol)
    if affine:
        _close(wv.grad.reshape(clients, ch), wr.grad, 3 * tol)
        _close(bv.grad.reshape(clients, ch), br.grad, 3 * tol)


def test_fused_group_norm_module_matches_torch():
    torch.manual_seed(0)
    m = torch.nn.GroupNorm(4, 64).to(DEV)
    with torch.no_grad():
        m.weight.uniform_(0.5, 1.5)
        m.bias.uniform_(-0.2, 0.2)
    f = torch.nn.GroupNorm(4, 64).to(DEV)
    f.load_state_dict(m.state_dict())
    assert ops.fuse_group_norm(f) == 1 and isinstance(f, FusedGroupNorm)
    x = torch.randn(6, 64, 9, 9, device=DEV)
    _close(f(x), m(x), 1e-4)


def test_engine_groupnorm_gpu_matches_cpu():
    """Client-batched engine with a GroupNorm net: GPU (HIP GN kernels, per-client affine from the
    arena) ≡ CPU reference engine after one local epoch (fp32 compute)."""
    import copy
    from fedml_amd.arguments import Arguments
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Conv2d(3, 16, 3, padding=1), torch.nn.GroupNorm(4, 16), torch.nn.ReLU(),
                                torch.nn.AdaptiveAvgPool2d(1), torch.nn.Flatten(), torch.nn.Linear(16, 5))
    C, n = 3, 32
    x, y = torch.randn(C * n, 3, 8, 8), torch.randint(0, 5, (C * n,))
    res = []
    for dev in ("cpu", DEV):
        args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": 0.05}})
        eng = ClientBatchEngine(copy.deepcopy(model).to(dev), C, dev, args, compute_dtype=None)
        flat = eng.layout.flatten(model.state_dict(), device=dev)
        eng.load_global(flat)
        eng.train(DeviceClientStore(x.to(dev), y.to(dev), [i * n for i in range(C)], [n] * C), torch.arange(C, device=dev),
                  1, 8, 0.05, shuffle=False)
        res.append((eng.params.cpu(), flat.cpu()))
        eng.close()
    (p0, f0), (p1, _) = res
    assert float((p0 - p1).norm() / (p0 - f0).norm()) < 1e-3
