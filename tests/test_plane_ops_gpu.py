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


def test_plane_bn_running_stats_and_arena_grads():
    """The engine's layout: γ, β, running mean / var and num_batches_tracked are strided rows of one parameter
    arena, γ/β gradients pre-assigned views of a gradient arena. The statistics kernel updates the running
    statistics in place (momentum, unbiased variance, active clients only) and the backward reduction
    accumulates dγ/dβ into the gradient arena (+=, autograd returns nothing for them)."""
    torch.manual_seed(2)
    C, Ch, B, HW, mom = 3, 16, 8, 6, 0.1
    P_ = 4 * Ch + 5
    arena = torch.rand(C, P_, device=DEV) + 0.5
    garena = torch.randn(C, P_, device=DEV)          # non-zero: the kernels must add, not store
    g0 = garena.clone()
    g = arena[:, 0:Ch].detach().requires_grad_(True)
    b = arena[:, Ch:2 * Ch].detach().requires_grad_(True)
    g.grad = garena[:, 0:Ch]
    b.grad = garena[:, Ch:2 * Ch]
    rm, rv, nbt = arena[:, 2 * Ch:3 * Ch], arena[:, 3 * Ch:4 * Ch], arena[:, 4 * Ch]
    rm0, rv0, nbt0 = rm.clone(), rv.clone(), nbt.clone()
    active = torch.tensor([1.0, 0.0, 1.0], device=DEV)
    x = (torch.randn(B, C * Ch, HW, HW, device=DEV) * 2 + 1).requires_grad_(True)
    y, _ = plane_ops.plane_batch_norm(x, g, b, C, 1e-5, relu=True, running=(rm, rv, nbt, mom, active))
    xr = x.detach().clone().requires_grad_(True)
    gr, br = g.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    rmr, rvr = rm0.reshape(-1).clone(), rv0.reshape(-1).clone()
    yr = torch.relu(F.batch_norm(xr, rmr, rvr, gr.reshape(-1), br.reshape(-1), True, mom, 1e-5))
    assert _rel(y, yr) < 2e-5
    on = active.view(C, 1) > 0
    assert _rel(rm, torch.where(on, rmr.view(C, Ch), rm0)) < 1e-5
    assert _rel(rv, torch.where(on, rvr.view(C, Ch), rv0)) < 1e-5
    assert torch.equal(nbt, nbt0 + active)
    gy = torch.randn_like(yr)
    (y * gy).sum().backward()
    (yr * gy).sum().backward()
    assert _rel(x.grad, xr.grad) < 1e-4
    assert _rel(garena[:, 0:Ch] - g0[:, 0:Ch], gr.grad) < 1e-4
    assert _rel(garena[:, Ch:2 * Ch] - g0[:, Ch:2 * Ch], br.grad) < 1e-5
    assert torch.equal(garena[:, 2 * Ch:], g0[:, 2 * Ch:])


def test_depthwise_wgrad_accumulates_into_arena():
    torch.manual_seed(3)
    C, Ch, B, K, H = 2, 8, 4, 3, 10
    P_ = Ch * K * K + 3
    arena = torch.randn(C, P_, device=DEV) * 0.3
    garena = torch.randn(C, P_, device=DEV)
    g0 = garena.clone()
    w = arena[:, 3:].view(C, Ch, 1, K, K).detach().requires_grad_(True)
    w.grad = garena[:, 3:].view(C, Ch, 1, K, K)
    wref = w.detach().clone().reshape(C * Ch, 1, K, K).requires_grad_(True)
    x = torch.randn(B, C * Ch, H, H, device=DEV)
    y = plane_ops.depthwise_conv2d(x, w, C, 1)
    yr = F.conv2d(x, wref, padding=K // 2, groups=C * Ch)
    gy = torch.randn_like(yr)
    (y * gy).sum().backward()
    (yr * gy).sum().backward()
    assert _rel((garena[:, 3:] - g0[:, 3:]).reshape(C * Ch, 1, K, K), wref.grad) < 2e-5
    assert torch.equal(garena[:, :3], g0[:, :3])


def test_mobilenet_step_native_within_fp32_envelope():
    """One MobileNet / CIFAR-10 step of 2 clients in the batched interpreter on the native kernels (plane
    depthwise + plane BN/ReLU + implicit-GEMM pointwise / stem convolutions: no MIOpen) and on PyTorch ops,
    both against a per-client fp64 nn.Module step. MobileNet at init sits on ReLU thresholds, so ANY fp32
    implementation's gradients move by ~1e-2 on some slots (mask flips; measured: PyTorch fp32 max 8.3e-3,
    median 3.9e-3). The native step must stay within 3× PyTorch fp32's own error on the same inputs (max and
    median over slots) and its logits within 1e-4 of fp64."""
    import copy
    from fedml_amd.core.arena import ParamLayout
    from fedml_amd.models.cv.mobilenet import mobilenet
    from fedml_amd.parallel import batched_nn
    torch.manual_seed(0)
    model = mobilenet(10).to(DEV)
    C, B = 2, 16
    layout = ParamLayout.from_module(model)
    x = torch.randn(C, B, 3, 32, 32, device=DEV)
    y = torch.randint(0, 10, (C, B), device=DEV)
    flat = layout.flatten(model.state_dict(), device=DEV)

    def run(native):
        saved = batched_nn._NATIVE_BCONV
        batched_nn._NATIVE_BCONV = native
        try:
            params = layout.alloc_stack(C, DEV)
            grads = layout.alloc_stack(C, DEV)
            params.copy_(flat.view(1, -1).expand(C, -1))
            views = {}
            for s in layout.slots:
                v = params[:, s.offset:s.offset + s.numel].view(C, *s.shape)
                if s.trainable:
                    v = v.detach().requires_grad_(True)
                    v.grad = grads[:, s.offset:s.offset + s.numel].view(C, *s.shape)
                views[s.key] = v
            out = batched_nn.BatchedInterpreter(model, layout, C).run(views, x, training=True)
            sum(F.cross_entropy(out[c], y[c]) for c in range(C)).backward()
            torch.cuda.synchronize()
            return out.detach(), grads.clone()
        finally:
            batched_nn._NATIVE_BCONV = saved

    o_nat, g_nat = run(True)
    o_t32, g_t32 = run(False)
    ref = torch.zeros(C, layout.size, dtype=torch.float64, device=DEV)
    o64 = []
    for c in range(C):
        m = copy.deepcopy(model).double().train()
        out = m(x[c].double())
        o64.append(out.detach())
        F.cross_entropy(out, y[c]).backward()
        for k, p in m.named_parameters():
            sl = layout.slot(k)
            ref[c, sl.offset:sl.offset + sl.numel] = p.grad.reshape(-1)
    assert _rel(o_nat, torch.stack(o64)) < 1e-4
    e_nat, e_t32 = [], []
    for sl in layout.slots:
        if sl.trainable:
            r = slice(sl.offset, sl.offset + sl.numel)
            e_nat.append(_rel(g_nat[:, r], ref[:, r]))
            e_t32.append(_rel(g_t32[:, r], ref[:, r]))
    med = lambda v: sorted(v)[len(v) // 2]   # noqa: E731
    assert max(e_nat) <= 3 * max(e_t32) + 1e-5, (max(e_nat), max(e_t32))
    assert med(e_nat) <= 3 * med(e_t32) + 1e-6, (med(e_nat), med(e_t32))


def test_mobilenet_engine_round_runs_native_and_learns(monkeypatch):
    """The engine's default (auto) path for MobileNet is the batched interpreter on the native kernels, and a
    few rounds on a learnable synthetic task lower the loss."""
    from fedml_amd.arguments import Arguments
    from fedml_amd.models.cv.mobilenet import mobilenet
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    torch.manual_seed(0)
    model = mobilenet(10)
    K, n, bs = 4, 32, 16
    yl = torch.randint(0, 10, (K * n,), device=DEV)
    xs = torch.randn(K * n, 3, 32, 32, device=DEV) * 0.5 + yl.view(-1, 1, 1, 1).float() / 5
    store = DeviceClientStore(xs, yl, [c * n for c in range(K)], [n] * K)
    args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": 0.05}})
    eng = ClientBatchEngine(model.to(DEV), K, DEV, args, compute_dtype=None)
    assert eng.interp is not None and not eng.sequential
    eng.load_global(eng.layout.flatten(model.state_dict(), device=DEV))
    losses = [float(eng.train(store, torch.arange(K, device=DEV), 1, bs, 0.05, shuffle=False)) for _ in range(4)]
    eng.close()
    assert losses[-1] < losses[0], losses
