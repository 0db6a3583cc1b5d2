"""Client-batched depthwise convolution and plane BatchNorm(+ReLU) kernels (csrc/plane_kernels.hip) against
plain PyTorch fp32 references of the same ops (grouped conv over the client-stacked channels, per-client
batch norm), and a MobileNet / CIFAR-10 round of the engine on the native plane + implicit-GEMM kernels
equal to the same round on PyTorch's (MIOpen) convolutions and batch norm."""
import copy

import pytest
import torch
import torch.nn.functional as F

from fedml_amd.ops import plane_ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@pytest.mark.parametrize("K,S,H", [(3, 1, 32), (3, 2, 32), (3, 2, 7), (5, 1, 16), (5, 2, 14), (3, 1, 2)])
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-5), (torch.bfloat16, 2e-2)])
def test_depthwise_conv_matches_grouped_conv(K, S, H, dtype, tol):
    torch.manual_seed(0)
    C, Ch, B = 3, 24, 5
    P_ = 7 + C * 0 + Ch * K * K + 5
    arena = torch.randn(C, P_, device=DEV) * 0.3
    w = arena[:, 7:7 + Ch * K * K].view(C, Ch, 1, K, K).detach().requires_grad_(True)
    wref = w.detach().clone().reshape(C * Ch, 1, K, K).requires_grad_(True)
    x = torch.randn(B, C * Ch, H, H, device=DEV)
    xn = x.to(dtype).requires_grad_(True)
    y = plane_ops.depthwise_conv2d(xn, w, C, S)
    xr = x.to(dtype).float().requires_grad_(True)
    yr = F.conv2d(xr, wref, stride=S, padding=K // 2, groups=C * Ch)
    assert y.shape == yr.shape and y.dtype == dtype
    assert _rel(y.float(), yr) < tol
    gy = torch.randn_like(yr)
    (y.float() * gy).sum().backward()
    (yr * gy).sum().backward()
    assert _rel(xn.grad.float(), xr.grad) < tol
    assert _rel(w.grad.reshape(C * Ch, 1, K, K), wref.grad) < tol


@pytest.mark.parametrize("relu", [False, True])
@pytest.mark.parametrize("HW,B", [(32, 8), (4, 64), (1, 16)])
def test_plane_batch_norm_matches_torch(relu, HW, B):
    torch.manual_seed(1)
    C, Ch = 4, 32
    x = (torch.randn(B, C * Ch, HW, HW, device=DEV) * 2 + 3).requires_grad_(True)
    arena = torch.rand(C, 2 * Ch + 9, device=DEV) + 0.5
    g = arena[:, 3:3 + Ch].detach().requires_grad_(True)
    b = arena[:, 3 + Ch:3 + 2 * Ch].detach().requires_grad_(True)
    y, (mean, var_b, n) = plane_ops.plane_batch_norm(x, g, b, C, 1e-5, relu=relu)
    xr = x.detach().clone().requires_grad_(True)
    gr = g.detach().clone().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = F.batch_norm(xr, None, None, gr.reshape(-1), br.reshape(-1), True, 0.0, 1e-5)
    if relu:
        yr = torch.relu(yr)
    assert _rel(y, yr) < 2e-5
    assert _rel(mean.reshape(-1), xr.detach().mean((0, 2, 3))) < 1e-5
    assert _rel(var_b.reshape(-1), xr.detach().var((0, 2, 3), unbiased=False)) < 1e-4 and n == B * HW * HW
    gy = torch.randn_like(yr)
    (y * gy).sum().backward()
    (yr * gy).sum().backward()
    assert _rel(x.grad, xr.grad) < 1e-4
    assert _rel(g.grad, gr.grad) < 1e-4 and _rel(b.grad, br.grad) < 1e-5


def test_mobilenet_round_native_equals_torch_engine(monkeypatch):
    """One local epoch of 10 MobileNet / CIFAR-10 clients: the native path (plane depthwise + plane BN/ReLU +
    implicit-GEMM pointwise / stem convolutions, no MIOpen convolution) equals the engine on PyTorch ops."""
    from fedml_amd.arguments import Arguments
    from fedml_amd.models.cv.mobilenet import mobilenet
    from fedml_amd.parallel import batched_nn
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    torch.manual_seed(0)
    model = mobilenet(10)
    K, n, bs = 10, 32, 16
    store = DeviceClientStore(torch.randn(K * n, 3, 32, 32, device=DEV), torch.randint(0, 10, (K * n,), device=DEV),
                              [c * n for c in range(K)], [n] * K)
    args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": 0.01, "weight_decay": 0.001,
                                      "client_exec": "batched"}})

    def run(native):
        monkeypatch.setattr(batched_nn, "_NATIVE_BCONV", native)
        eng = ClientBatchEngine(copy.deepcopy(model).to(DEV), K, DEV, args, compute_dtype=None)
        assert eng.interp is not None and not eng.sequential
        eng.load_global(eng.layout.flatten(model.state_dict(), device=DEV))
        eng.train(store, torch.arange(K, device=DEV), 1, bs, 0.01, shuffle=False)
        torch.cuda.synchronize()
        out = eng.params.clone()
        eng.close()
        return out

    from fedml_amd.core.arena import ParamLayout
    init = ParamLayout.from_module(model).flatten(model.state_dict(), device=DEV)
    nat, ref = run(True), run(False)
    assert torch.isfinite(nat).all()
    # relative to the round's update (the parameters themselves are much larger than one epoch's change)
    err = float((nat - ref).double().norm() / (ref - init).double().norm())
    assert err < 1e-3, err
