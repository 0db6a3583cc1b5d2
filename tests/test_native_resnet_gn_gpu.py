"""Native ResNet-GN step (parallel/native_resnet_gn.py, csrc/gnh_kernels.hip) against PyTorch: the NHWC GroupNorm /
max-pool kernels against torch fp32 ops, and one whole client-batched step against each client's own fp64 torch
backward on its valid images (heterogeneous counts, an idle client) — the model of the reference's fed_CIFAR-100
benchmark (`model/cv/resnet_gn.py:187-239`)."""
import copy

import pytest
import torch
import torch.nn.functional as F

from fedml_amd.core.arena import ParamLayout
from fedml_amd.models.cv.resnet_gn import resnet18
from fedml_amd.ops import nn_ops
from fedml_amd.parallel.native_resnet_gn import NativeGNResNetStep

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("hw,ch,groups", [(36, 64, 2), (9, 128, 4), (1, 512, 16), (144, 64, 2)])
@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, False)])
def test_gnh_fwd_bwd_match_torch(hw, ch, groups, relu, res):
    torch.manual_seed(0)
    C, N = 3, 5
    nimg = torch.tensor([5, 2, 0], dtype=torch.int32, device=DEV)
    x = torch.randn(C, N, hw, ch, device=DEV)
    r = torch.randn(C, N, hw, ch, device=DEV) if res else None
    arena = torch.randn(C, 2 * ch + 8, device=DEV)
    arena[:, :ch] = arena[:, :ch].abs() + 0.5
    out = torch.zeros_like(x)
    ms = torch.zeros(C, N, groups, 2, device=DEV)
    nn_ops.gnh_fwd(x, r, out, ms, arena, 0, ch, C, N, hw, ch, groups, 1e-5, relu, nimg=nimg)
    go = torch.randn_like(x)
    dx = torch.zeros_like(x)
    pscr = torch.zeros(C, N, 2, ch, device=DEV)
    garena = torch.zeros_like(arena)
    nn_ops.gnh_bwd(x, go, out if relu else None, dx, ms, pscr, arena, 0, C, N, hw, ch, groups, nimg=nimg)
    nn_ops.gnh_param_reduce(pscr, garena, 0, ch, C, N, ch, nimg=nimg)
    torch.cuda.synchronize()
    for c in range(C):
        n = int(nimg[c])
        if n == 0:
            assert float(garena[c].abs().max()) == 0.0
            continue
        xc = x[c, :n].permute(0, 2, 1).contiguous().requires_grad_(True)      # [n, ch, hw]
        w, b = arena[c, :ch].clone().requires_grad_(True), arena[c, ch:2 * ch].clone().requires_grad_(True)
        y = F.group_norm(xc, groups, w, b, 1e-5)
        if res:
            y = y + r[c, :n].permute(0, 2, 1)
        if relu:
            y = torch.relu(y)
        assert torch.allclose(out[c, :n].permute(0, 2, 1), y, atol=2e-5, rtol=1e-4)
        y.backward(go[c, :n].permute(0, 2, 1))
        assert torch.allclose(dx[c, :n].permute(0, 2, 1), xc.grad, atol=5e-5, rtol=1e-3), \
            float((dx[c, :n].permute(0, 2, 1) - xc.grad).abs().max())
        assert torch.allclose(garena[c, :ch], w.grad, atol=1e-3, rtol=1e-4)
        assert torch.allclose(garena[c, ch:2 * ch], b.grad, atol=1e-3, rtol=1e-4)


def test_maxpool_fwd_bwd_match_torch():
    torch.manual_seed(1)
    C, N, H, W, ch = 2, 3, 12, 12, 64
    x = torch.randn(C, N, H, W, ch, device=DEV)
    Ho = Wo = 6
    y = torch.zeros(C, N, Ho, Wo, ch, device=DEV)
    idx = torch.zeros(C, N, Ho, Wo, ch, dtype=torch.uint8, device=DEV)
    nn_ops.maxpool_fwd(x, y, idx, C, N, H, W, ch, Ho, Wo, 3, 2, 1)
    gy = torch.randn_like(y)
    gx = torch.zeros_like(x)
    nn_ops.maxpool_bwd(gy, idx, gx, C, N, H, W, ch, Ho, Wo, 3, 2, 1)
    xt = x.reshape(C * N, H, W, ch).permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    yt = F.max_pool2d(xt, 3, 2, 1)
    yt.backward(gy.reshape(C * N, Ho, Wo, ch).permute(0, 3, 1, 2))
    assert torch.equal(y.reshape(C * N, Ho, Wo, ch).permute(0, 3, 1, 2), yt)
    assert torch.allclose(gx.reshape(C * N, H, W, ch).permute(0, 3, 1, 2), xt.grad, atol=1e-6)


def test_native_gn_step_matches_fp64_torch():
    """Clients with 8, 5 and 0 valid images: every client's gradients equal its own fp64 torch step on its valid
    images; the idle client gets exactly zero gradients."""
    torch.manual_seed(0)
    model = resnet18(100)
    layout = ParamLayout.from_module(model)
    C, N = 3, 8
    counts = [8, 5, 0]
    flat = layout.flatten(model.state_dict()).to(DEV)
    arena = flat.view(1, -1).repeat(C, 1).contiguous()
    garena = torch.zeros_like(arena)
    x = torch.randn(C, N, 3, 24, 24, device=DEV)
    y = torch.randint(0, 100, (C, N), device=DEV)
    mask = torch.arange(N, device=DEV).view(1, -1) < torch.tensor(counts, device=DEV).view(-1, 1)
    row_scale = mask.float() / torch.tensor([max(1, b) for b in counts], device=DEV).view(-1, 1)
    active = torch.tensor([1.0 if b else 0.0 for b in counts], device=DEV)
    nimg = torch.tensor(counts, dtype=torch.int32, device=DEV)
    step = NativeGNResNetStep(model, layout, C, DEV)
    loss = float(step.step(arena, garena, x, y, row_scale, active, nimg=nimg))
    torch.cuda.synchronize()
    ref_loss = 0.0
    for c, b in enumerate(counts):
        g = garena[c]
        if b == 0:
            assert float(g.abs().max()) == 0.0
            continue
        m = copy.deepcopy(model).double()
        lo = F.cross_entropy(m(x[c, :b].cpu().double()), y[c, :b].cpu())
        lo.backward()
        ref_loss += float(lo)
        for name, p in m.named_parameters():
            s = layout.slot(name)
            got = g[s.offset:s.offset + s.numel].cpu().double()
            r = p.grad.reshape(-1)
            err = float((got - r).norm() / r.norm().clamp_min(1e-30))
            assert err < 5e-3, (c, name, err)
    assert abs(loss - ref_loss) / ref_loss < 1e-5


def test_engine_picks_native_gn_and_learns():
    from fedml_amd.arguments import Arguments
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    torch.manual_seed(0)
    model = resnet18(100).to(DEV)
    args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": 0.05}})
    eng = ClientBatchEngine(model, 4, DEV, args, compute_dtype=None)
    assert eng.executor == "native" and isinstance(eng.native_step, NativeGNResNetStep)
    counts = [40, 33, 20, 0]
    n = sum(counts)
    store = DeviceClientStore(torch.randn(n, 3, 24, 24, device=DEV), torch.randint(0, 100, (n,), device=DEV),
                              [0, 40, 73, 93], counts)
    eng.load_global(eng.layout.flatten(model.state_dict(), device=DEV))
    first = None
    for r in range(6):
        loss = float(eng.train(store, torch.arange(4, device=DEV), 1, 10, 0.05, shuffle=False))
        first = loss if first is None else first
    assert torch.isfinite(eng.params).all() and loss < first
    eng.close()
