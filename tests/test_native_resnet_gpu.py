"""Native client-batched ResNet step (HIP conv/BN kernels) vs the fp32 PyTorch reference of the
same per-client computation (sequential single-client models)."""
import copy

import pytest
import torch

from fedml_amd.core.arena import ParamLayout
from fedml_amd.models.cv.resnet import BasicBlock, Bottleneck, ResNet, resnet56
from fedml_amd.parallel.native_resnet import NativeResNetStep

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _reference_grads(model, layout, flat, x, y, autocast=False):
    """Per-client fp32 (or bf16-autocast) forward/backward; returns (loss_sum, grads [C, P])."""
    C = x.shape[0]
    grads = torch.zeros(C, layout.size, device=DEV)
    loss_sum = 0.0
    for c in range(C):
        m = copy.deepcopy(model).to(DEV).float()
        m.load_state_dict(layout.unflatten(flat))
        m.train()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            out = m(x[c])
        loss = torch.nn.functional.cross_entropy(out.float(), y[c])
        loss.backward()
        loss_sum += float(loss.detach())
        sd = {k: p.grad for k, p in m.named_parameters()}
        for s in layout.slots:
            if s.key in sd:
                grads[c, s.offset:s.offset + s.numel] = sd[s.key].reshape(-1)
    return loss_sum, grads


@pytest.mark.parametrize("builder,hw", [
    (lambda: ResNet(Bottleneck, [1, 1, 1], 10), 16),
    (lambda: ResNet(BasicBlock, [2, 1, 1], 10), 16),
    (lambda: ResNet(Bottleneck, [2, 2, 2], 100), 32),
])
def test_native_step_matches_reference(builder, hw):
    torch.manual_seed(0)
    model = builder()
    layout = ParamLayout.from_module(model)
    C, N = 3, 16
    flat = layout.flatten(model.state_dict()).to(DEV)
    arena = flat.view(1, -1).repeat(C, 1).contiguous()
    garena = torch.zeros_like(arena)
    x = torch.randn(C, N, 3, hw, hw, device=DEV)
    y = torch.randint(0, model.fc.out_features, (C, N), device=DEV)
    row_scale = torch.full((C, N), 1.0 / N, device=DEV)
    active = torch.ones(C, device=DEV)
    step = NativeResNetStep(model, layout, C, DEV, dtype=torch.bfloat16)
    loss = float(step.step(arena, garena, x, y, row_scale, active))
    torch.cuda.synchronize()
    ref_loss, ref = _reference_grads(model, layout, flat, x, y)
    _, ref_bf16 = _reference_grads(model, layout, flat, x, y, autocast=True)
    assert abs(loss - ref_loss) / ref_loss < 2e-2, (loss, ref_loss)
    # Small-batch random-init ResNets are ill-conditioned: PyTorch's own bf16 autocast moves
    # the gradients by 20-45 % here. The native path (bf16 activations, fp32 BN/accumulation)
    # must be within the same error envelope as autocast and point the same way.
    bad = []
    for s in layout.slots:
        if not s.trainable:
            continue
        g = garena[:, s.offset:s.offset + s.numel]
        r = ref[:, s.offset:s.offset + s.numel]
        a = ref_bf16[:, s.offset:s.offset + s.numel]
        err = float((g - r).norm() / r.norm().clamp_min(1e-8))
        err_ac = float((a - r).norm() / r.norm().clamp_min(1e-8))
        cos = float((g * r).sum() / (g.norm() * r.norm()).clamp_min(1e-12))
        cos_ac = float((a * r).sum() / (a.norm() * r.norm()).clamp_min(1e-12))
        if err > 2.0 * err_ac + 0.05 or cos < min(0.9, cos_ac - 0.1):
            bad.append((s.key, round(err, 4), round(err_ac, 4), round(cos, 4)))
    assert not bad, bad[:8]
    # running statistics updated like torch (momentum 0.1, unbiased var)
    s = layout.slot("bn1.running_mean")
    m = copy.deepcopy(model).to(DEV)
    m.train()
    m(x[0])
    assert torch.allclose(arena[0, s.offset:s.offset + s.numel], m.bn1.running_mean, atol=2e-2, rtol=5e-2)


def test_native_resnet56_engine_round():
    from fedml_amd.arguments import Arguments
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    torch.manual_seed(0)
    model = resnet56(100)
    args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": 0.05}})
    eng = ClientBatchEngine(model.to(DEV), 4, DEV, args, compute_dtype=torch.bfloat16)
    assert eng.native_step is not None
    flat = eng.layout.flatten(model.state_dict(), device=DEV)
    eng.load_global(flat)
    n = 4 * 64
    store = DeviceClientStore(torch.randn(n, 3, 32, 32, device=DEV), torch.randint(0, 100, (n,), device=DEV),
                              [0, 64, 128, 192], [64] * 4)
    losses = []
    for _ in range(3):
        losses.append(float(eng.train(store, torch.arange(4, device=DEV), 1, 32, 0.05, shuffle=False)))
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < losses[0]   # memorising the same data → loss decreases


@pytest.mark.parametrize("ch,hw,stride", [(16, 32, 1), (32, 16, 1), (64, 8, 1), (16, 16, 1), (32, 32, 2),
                                         (64, 16, 2)])
def test_conv3x3_kernels_vs_fp32_reference(ch, hw, stride):
    """LDS-tiled 3×3 kernels against torch fp32 convolutions of the same bf16 operands, and against
    the generic implicit-GEMM kernels (forward / backward-data agree with the latter to a bf16 ulp)."""
    from fedml_amd.ops import nn_ops
    torch.manual_seed(0)
    C, N, bf = 3, 8, torch.bfloat16
    K = 9 * ch
    ldk = (K + 31) // 32 * 32 + 8
    x = torch.randn(C, N, hw, hw, ch, device=DEV).to(bf)
    wpk = torch.zeros(C, ch, ldk, device=DEV)
    wpk[:, :, :K] = torch.randn(C, ch, K, device=DEV) * 0.1
    wpk = wpk.to(bf).contiguous()
    s = torch.rand(C, ch, device=DEV) + 0.5
    t = torch.randn(C, ch, device=DEV) * 0.1
    wt = wpk[:, :, :K].float().view(C, ch, 3, 3, ch).permute(0, 1, 4, 2, 3)  # [C][co][ci][kh][kw]
    # the same buffer read as the backward packing Wb[ci][tap·Cout + co] → W[co][ci][kh][kw]
    wt_b = wpk[:, :, :K].float().view(C, ch, 3, 3, ch).permute(0, 4, 1, 2, 3)

    def rel(a, b):
        return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))

    ho = hw // stride
    # forward: y = conv(relu(x·s + t)), BN statistics (Σy, Σy²)
    y3 = torch.zeros(C, N, ho, ho, ch, device=DEV, dtype=bf)
    st3 = torch.zeros(C, ch, 2, device=DEV)
    nn_ops.conv3x3_fwd(x, wpk, ch * ldk, s, t, y3, st3, C, N, hw, hw, ch, ch, ldk, stride)
    yg = torch.zeros_like(y3)
    stg = torch.zeros_like(st3)
    nn_ops.conv_fwd(x, wpk, ch * ldk, s, t, yg, stg, C, N, hw, hw, ch, ch, 3, 3, stride, 1, ho, ho, ldk, 1)
    torch.cuda.synchronize()
    assert rel(y3, yg) < 5e-3  # same operands; FMA contraction may differ by a bf16 ulp
    for c in range(C):
        xa = torch.relu(x[c].float() * s[c] + t[c]).to(bf).float().permute(0, 3, 1, 2)
        ref = torch.nn.functional.conv2d(xa, wt[c], padding=1, stride=stride).permute(0, 2, 3, 1)
        assert rel(y3[c], ref) < 1e-2
        assert rel(st3[c, :, 0], y3[c].float().sum((0, 1, 2))) < 1e-4
    # backward-data with the ReLU-mask epilogue
    g = torch.randn(C, N, ho, ho, ch, device=DEV).to(bf)
    yv = torch.randn(C, N, ho, ho, ch, device=DEV).to(bf)
    al, be = torch.rand(C, ch, device=DEV), torch.randn(C, ch, device=DEV) * 0.1
    ga = torch.randn(C, ch, device=DEV) * 0.01
    ex = torch.randn(C, N, hw, hw, ch, device=DEV).to(bf)
    dx = torch.zeros_like(ex)
    st = torch.zeros(C, ch, 3, device=DEV)
    nn_ops.conv3x3_bwd_data(g, yv, al, be, ga, wpk, ch * ldk, dx, ex, s, t, st, C, N, hw, hw, ch, ch, ldk, stride)
    dxg = torch.zeros_like(ex)
    stg = torch.zeros_like(st)
    nn_ops.conv_bwd_data(g, yv, al, be, ga, wpk, ch * ldk, dxg, nn_ops.EPI_MASK, ex, s, t, None, None, None, stg,
                         C, N, ho, ho, ch, ch, 3, 3, stride, 1, hw, hw, ldk, 1)
    torch.cuda.synchronize()
    assert rel(dx, dxg) < 5e-3
    for c in range(C):
        dy = (al[c] * g[c].float() + be[c] * yv[c].float() + ga[c]).to(bf).float().permute(0, 3, 1, 2)
        ref = torch.nn.grad.conv2d_input((N, ch, hw, hw), wt_b[c], dy, padding=1, stride=stride).permute(0, 2, 3, 1)
        mask = (ex[c].float() * s[c] + t[c]) > 0
        assert rel(dx[c], ref * mask) < 1e-2
    # weight gradient
    P = ch * ch * 9 + 64
    garena = torch.zeros(C, P, device=DEV)
    scratch = torch.zeros(C * ch * K, device=DEV)
    nn_ops.conv3x3_wgrad(g, yv, al, be, ga, x, s, t, garena, 16, C, N, hw, hw, ch, ch, ch, scratch, stride)
    torch.cuda.synchronize()
    assert float(scratch.abs().max()) == 0.0  # scatter pass leaves the scratch zeroed
    for c in range(C):
        dy = (al[c] * g[c].float() + be[c] * yv[c].float() + ga[c]).to(bf).float().permute(0, 3, 1, 2)
        xa = torch.relu(x[c].float() * s[c] + t[c]).to(bf).float().permute(0, 3, 1, 2)
        ref = torch.nn.grad.conv2d_weight(xa, (ch, ch, 3, 3), dy, padding=1, stride=stride)
        assert rel(garena[c, 16:16 + ch * ch * 9], ref.reshape(-1)) < 1e-4


@pytest.mark.parametrize("ch,hw,N", [(16, 32, 8), (32, 16, 8), (64, 32, 4), (64, 8, 16)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("y2", [False, True])
def test_conv3x3_bwd_data_block_epilogue(ch, hw, N, dtype, y2):
    """3×3 tile kernel with the block epilogue (a basic block's first conv): dx' = (convᵀ(dy) + e_add)·[e_x > 0]
    and the statistics (Σdx', Σdx'·y1, Σdx'·y2) against torch fp32 of the same operands, and against the
    generic implicit-GEMM kernel's EPI_BLOCK."""
    from fedml_amd.ops import nn_ops
    torch.manual_seed(3)
    C, dt = 3, dtype
    K = 9 * ch
    ldk = (K + 31) // 32 * 32 + 8
    wpk = torch.zeros(C, ch, ldk, device=DEV)
    wpk[:, :, :K] = torch.randn(C, ch, K, device=DEV) * 0.1
    wpk = wpk.to(dt).contiguous()
    wt_b = wpk[:, :, :K].float().view(C, ch, 3, 3, ch).permute(0, 4, 1, 2, 3)
    g = torch.randn(C, N, hw, hw, ch, device=DEV).to(dt)
    yv = torch.randn(C, N, hw, hw, ch, device=DEV).to(dt)
    al, be = torch.rand(C, ch, device=DEV), torch.randn(C, ch, device=DEV) * 0.1
    ga = torch.randn(C, ch, device=DEV) * 0.01
    ex = torch.relu(torch.randn(C, N, hw, hw, ch, device=DEV)).to(dt)      # block input (post-ReLU)
    ea = torch.randn(C, N, hw, hw, ch, device=DEV).to(dt)                  # shortcut gradient
    e1 = torch.randn(C, N, hw, hw, ch, device=DEV).to(dt)
    e2 = torch.randn(C, N, hw, hw, ch, device=DEV).to(dt) if y2 else None
    dx = torch.zeros_like(ex)
    st = torch.zeros(C, ch, 3, device=DEV)
    nn_ops.conv3x3_bwd_data_block(g, yv, al, be, ga, wpk, ch * ldk, dx, ex, ea, e1, e2, st, C, N, hw, hw, ch, ch, ldk)
    dxg = torch.zeros_like(ex)
    stg = torch.zeros_like(st)
    nn_ops.conv_bwd_data(g, yv, al, be, ga, wpk, ch * ldk, dxg, nn_ops.EPI_BLOCK, ex, None, None, ea, e1, e2, stg,
                         C, N, hw, hw, ch, ch, 3, 3, 1, 1, hw, hw, ldk, 1)
    torch.cuda.synchronize()

    def rel(a, b):
        return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))

    tol = 1e-2 if dt == torch.bfloat16 else 1e-5
    assert rel(dx, dxg) < (5e-3 if dt == torch.bfloat16 else 1e-5)
    for c in range(C):
        dy = (al[c] * g[c].float() + be[c] * yv[c].float() + ga[c]).to(dt).float().permute(0, 3, 1, 2)
        ref = torch.nn.grad.conv2d_input((N, ch, hw, hw), wt_b[c], dy, padding=1).permute(0, 2, 3, 1)
        ref = (ref + ea[c].float()) * (ex[c].float() > 0)
        assert rel(dx[c], ref) < tol
        d = dx[c].float()
        assert rel(st[c, :, 0], d.sum((0, 1, 2))) < 1e-4
        assert rel(st[c, :, 1], (d * e1[c].float()).sum((0, 1, 2))) < 1e-4
        if y2:
            assert rel(st[c, :, 2], (d * e2[c].float()).sum((0, 1, 2))) < 1e-4
        else:
            assert float(st[c, :, 2].abs().max()) == 0.0
        assert rel(st[c], stg[c]) < (1e-2 if dt == torch.bfloat16 else 1e-5)


@pytest.mark.parametrize("cin,cout,hw", [(16, 64, 32), (64, 16, 32), (32, 128, 16), (128, 32, 16), (64, 256, 8),
                                         (256, 64, 8), (64, 64, 8)])
@pytest.mark.parametrize("pro", [False, True])
def test_conv1x1_wgrad_vs_fp32_reference(cin, cout, hw, pro):
    from fedml_amd.ops import nn_ops
    torch.manual_seed(1)
    C, N, bf = 3, 8, torch.bfloat16
    x = torch.randn(C, N, hw, hw, cin, device=DEV).to(bf)
    g = torch.randn(C, N, hw, hw, cout, device=DEV).to(bf)
    yv = torch.randn(C, N, hw, hw, cout, device=DEV).to(bf)
    al, be = torch.rand(C, cout, device=DEV), torch.randn(C, cout, device=DEV) * 0.1
    ga = torch.randn(C, cout, device=DEV) * 0.01
    s = torch.rand(C, cin, device=DEV) + 0.5 if pro else None
    t = torch.randn(C, cin, device=DEV) * 0.1 if pro else None
    garena = torch.zeros(C, cin * cout + 48, device=DEV)
    M = N * hw * hw
    nn_ops.conv1x1_wgrad(g, yv, al, be, ga, x, s, t, garena, 16, C, M, cin, cout, 512)
    torch.cuda.synchronize()
    for c in range(C):
        dy = (al[c] * g[c].float() + be[c] * yv[c].float() + ga[c]).to(bf).float().reshape(-1, cout)
        xa = x[c].float()
        if pro:
            xa = torch.relu(xa * s[c] + t[c]).to(bf).float()
        ref = dy.t() @ xa.reshape(-1, cin)
        got = garena[c, 16:16 + cin * cout].view(cout, cin)
        assert float((got - ref).norm() / ref.norm()) < 1e-4


@pytest.mark.parametrize("cin,cout,epi", [(16, 64, 2), (32, 128, 2), (64, 256, 2), (64, 16, 3), (128, 32, 3),
                                          (256, 64, 3), (16, 16, 3), (64, 32, 3), (128, 64, 3)])
@pytest.mark.parametrize("M,ppw", [(8 * 16 * 16, 512), (5 * 7 * 7, 64)])
@pytest.mark.parametrize("two_pass", [False, True])
def test_conv1x1_bwd_fused_vs_fp32_reference(cin, cout, epi, M, ppw, two_pass):
    """Fused 1×1 data+weight gradient vs the fp32 reference of both products and the epilogue."""
    from fedml_amd.ops import nn_ops
    torch.manual_seed(2)
    C, bf = 3, torch.bfloat16
    rel = lambda a, b: float((a - b).norm() / b.norm().clamp_min(1e-12))
    g = torch.randn(C, M, cout, device=DEV).to(bf)
    yv = torch.randn(C, M, cout, device=DEV).to(bf)
    al, be = torch.rand(C, cout, device=DEV), torch.randn(C, cout, device=DEV) * 0.1
    ga = torch.randn(C, cout, device=DEV) * 0.01
    W = (torch.randn(C, cout, cin, device=DEV) / cin ** 0.5).to(bf)
    ld = (cout + 31) // 32 * 32 + 8
    wb = torch.zeros(C, cin * ld + 64, device=DEV, dtype=bf)
    wb[:, :cin * ld].view(C, cin, ld)[:, :, :cout] = W.transpose(1, 2)
    e_x = torch.randn(C, M, cin, device=DEV).to(bf)
    s = t = e_add = e_y1 = e_y2 = None
    if epi == 2:
        s, t = torch.rand(C, cin, device=DEV) + 0.5, torch.randn(C, cin, device=DEV) * 0.1
    else:
        e_add, e_y1, e_y2 = (torch.randn(C, M, cin, device=DEV).to(bf) for _ in range(3))
    out = torch.empty(C, M, cin, device=DEV, dtype=bf)
    stats = torch.zeros(C, cin, 3, device=DEV)
    garena = torch.zeros(C, cin * cout + 48, device=DEV)
    part = torch.full((nn_ops.conv1x1_bwd_fused_scratch(C, M, cin, cout, ppw),), float("nan"),
                      device=DEV) if two_pass else None
    nn_ops.conv1x1_bwd_fused(g, yv, al, be, ga, wb, wb.stride(0), ld, e_x, s, t, e_add, e_y1, e_y2, out, stats,
                             garena, 16, C, M, cin, cout, epi, ppw, part)
    torch.cuda.synchronize()
    for c in range(C):
        dy = (al[c] * g[c].float() + be[c] * yv[c].float() + ga[c]).to(bf).float()
        dx = (dy @ W[c].float()).to(bf).float()
        xr = e_x[c].float()
        if epi == 2:
            gp = torch.where(xr * s[c] + t[c] > 0, dx, torch.zeros_like(dx)).to(bf).float()
            st = torch.stack([gp.sum(0), (gp * xr).sum(0)], -1)
            act = torch.relu(xr * s[c] + t[c]).to(bf).float()
        else:
            gp = torch.where(xr > 0, dx + e_add[c].float(), torch.zeros_like(dx)).to(bf).float()
            st = torch.stack([gp.sum(0), (gp * e_y1[c].float()).sum(0), (gp * e_y2[c].float()).sum(0)], -1)
            act = xr
        assert rel(out[c].float(), gp) < 1e-2
        assert rel(stats[c, :, :st.shape[-1]], st) < 1e-2
        ref_dw = dy.t() @ act
        assert rel(garena[c, 16:16 + cin * cout].view(cout, cin), ref_dw) < 1e-4
    assert float(garena[:, :16].abs().max()) == 0.0 and float(garena[:, 16 + cin * cout:].abs().max()) == 0.0


@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_hip_graph_step_matches_eager(momentum):
    """The captured local step (zero grads → forward/backward kernels → fused optimizer) leaves the
    arenas where eager launches do; BN running statistics are not double-counted by the capture."""
    from fedml_amd.arguments import Arguments
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    torch.manual_seed(0)
    model = ResNet(Bottleneck, [1, 1, 1], 10)
    n = 3 * 64
    store = DeviceClientStore(torch.randn(n, 3, 16, 16, device=DEV), torch.randint(0, 10, (n,), device=DEV),
                              [0, 64, 128], [64] * 3)
    outs = []
    for graphs in (False, True):
        args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": 0.05, "momentum": momentum}})
        eng = ClientBatchEngine(copy.deepcopy(model).to(DEV), 3, DEV, args, compute_dtype=torch.bfloat16)
        eng.use_graphs = graphs
        eng.load_global(eng.layout.flatten(model.state_dict(), device=DEV))
        loss = float(eng.train(store, torch.arange(3, device=DEV), 1, 32, 0.05, shuffle=False))
        torch.cuda.synchronize()
        outs.append((loss, eng.params.clone()))
        if graphs:
            assert len(eng._graphs) >= 1
    (l0, p0), (l1, p1) = outs
    assert abs(l0 - l1) / abs(l0) < 1e-2
    # two local steps of SGD from identical weights: parameters agree up to atomics ordering noise
    assert float((p0 - p1).norm() / p0.norm()) < 1e-3


@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_multistream_graph_seq_step_matches_eager(momentum, monkeypatch):
    """Wide conv nets (ResNet-18 with the native kernels switched off: FEDML_AMD_NATIVE_CONV=0) run per client; the captured multi-stream step (C client branches
    on forked HIP streams + fused optimizer, one replay) matches the eager one-client-after-another
    step, BN running statistics included. fp32 compute and a small learning rate: MIOpen's
    backward kernels are not bitwise deterministic, and at lr 0.05 two EAGER runs of ResNet-18 already
    differ by ~1 % of the update (bf16: ~5 %) — measured, scripts/dbg_seqgraph.py."""
    from fedml_amd.arguments import Arguments
    from fedml_amd.models.cv.resnet import resnet18_cifar
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    monkeypatch.setenv("FEDML_AMD_NATIVE_CONV", "0")
    torch.manual_seed(0)
    model = resnet18_cifar(10)
    C, n = 3, 128
    store = DeviceClientStore(torch.randn(C * n, 3, 16, 16, device=DEV), torch.randint(0, 10, (C * n,), device=DEV),
                              [i * n for i in range(C)], [n] * C)
    outs = []
    for graphs in (False, True):
        args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": 1e-3, "momentum": momentum,
                                          "client_exec": "sequential"}})
        eng = ClientBatchEngine(copy.deepcopy(model).to(DEV), C, DEV, args, compute_dtype=None)
        assert eng.sequential and eng.tf is None
        eng.use_graphs = graphs
        eng.load_global(eng.layout.flatten(model.state_dict(), device=DEV))
        loss = float(eng.train(store, torch.arange(C, device=DEV), 1, 32, 1e-3, shuffle=False))
        torch.cuda.synchronize()
        outs.append((loss, eng.params.clone()))
        if graphs:
            assert any(isinstance(v, tuple) for v in eng._graphs.values())
        eng.close()
    (l0, p0), (l1, p1) = outs
    init = ParamLayout.from_module(model).flatten(model.state_dict(), device=DEV)
    assert abs(l0 - l1) / abs(l0) < 1e-3
    assert float((p0 - p1).norm() / (p0 - init).norm()) < 1e-3


def test_padding_slot_keeps_native_graph_path():
    """A GPU hosting fewer clients than C (8-GPU run: 12 of 13 slots valid) stays on the captured
    native step: the padding slot is inactive (unchanged parameters), the valid clients match eager."""
    from fedml_amd.arguments import Arguments
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    torch.manual_seed(0)
    model = ResNet(Bottleneck, [1, 1, 1], 10)
    n = 3 * 64
    store = DeviceClientStore(torch.randn(n, 3, 16, 16, device=DEV), torch.randint(0, 10, (n,), device=DEV),
                              [0, 64, 128], [64] * 3)
    valid = torch.tensor([True, True, False], device=DEV)
    outs = []
    for graphs in (False, True):
        args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": 0.05}})
        eng = ClientBatchEngine(copy.deepcopy(model).to(DEV), 3, DEV, args, compute_dtype=torch.bfloat16)
        assert eng.native_step is not None
        eng.use_graphs = graphs
        flat = eng.layout.flatten(model.state_dict(), device=DEV)
        eng.load_global(flat)
        eng.train(store, torch.arange(3, device=DEV), 1, 32, 0.05, shuffle=False, valid_slots=valid)
        torch.cuda.synchronize()
        outs.append(eng.params.clone())
        if graphs:
            assert len(eng._graphs) >= 1        # captured despite the padding slot
        assert torch.equal(eng.params[2], flat)  # padding slot untouched
        eng.close()
    p0, p1 = outs
    assert float((p0[:2] - p1[:2]).norm() / p0[:2].norm()) < 1e-3


def test_conv_weight_shadow_matches_autocast_path(monkeypatch):
    """Per-client path with bf16 channels-last conv-weight leaves from the packed shadow ≡ the
    autocast path (same bf16 rounding of the fp32 masters; only MIOpen's algorithm choice differs)."""
    from fedml_amd.arguments import Arguments
    from fedml_amd.models.cv.resnet import resnet18_cifar
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    monkeypatch.setenv("FEDML_AMD_NATIVE_CONV", "0")   # the per-client library path (ResNet-18 is native now)
    torch.manual_seed(0)
    model = resnet18_cifar(10)
    C, n = 2, 64
    store = DeviceClientStore(torch.randn(C * n, 3, 16, 16, device=DEV), torch.randint(0, 10, (C * n,), device=DEV),
                              [i * n for i in range(C)], [n] * C)
    outs = []
    for shadow in ("0", "1"):
        monkeypatch.setenv("FEDML_AMD_SEQ_CONV_SHADOW", shadow)
        args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": 1e-3,
                                          "client_exec": "sequential"}})
        eng = ClientBatchEngine(copy.deepcopy(model).to(DEV), C, DEV, args, compute_dtype=torch.bfloat16)
        eng.load_global(eng.layout.flatten(model.state_dict(), device=DEV))
        loss = float(eng.train(store, torch.arange(C, device=DEV), 1, 32, 1e-3, shuffle=False))
        torch.cuda.synchronize()
        outs.append((loss, eng.params.clone()))
        if shadow == "1":
            assert eng._cshadow_views      # the shadow path ran
        eng.close()
    (l0, p0), (l1, p1) = outs
    init = ParamLayout.from_module(model).flatten(model.state_dict(), device=DEV)
    assert abs(l0 - l1) / abs(l0) < 1e-2
    assert float((p0 - p1).norm() / (p0 - init).norm()) < 5e-2


def test_seq_graph_reads_the_rounds_class_weights(monkeypatch):
    """S-FedAvg's class-balanced CE on the captured per-client path: the class-weight table changes
    every round; the captured graph must read THIS round's table (one persistent engine buffer, refilled in place),
    so three rounds with different tables give the same parameters replayed as run eagerly."""
    from fedml_amd.arguments import Arguments
    from fedml_amd.models.cv.resnet import resnet18_cifar
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    monkeypatch.setenv("FEDML_AMD_NATIVE_CONV", "0")
    torch.manual_seed(0)
    model = resnet18_cifar(10)
    C, n = 2, 64
    store = DeviceClientStore(torch.randn(C * n, 3, 16, 16, device=DEV), torch.randint(0, 10, (C * n,), device=DEV),
                              [i * n for i in range(C)], [n] * C)
    g = torch.Generator().manual_seed(3)
    tables = [torch.rand(C, 10, generator=g) * 3 + 0.1 for _ in range(3)]
    outs = []
    for graphs in (False, True):
        args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": 1e-3,
                                          "client_exec": "sequential"}})
        eng = ClientBatchEngine(copy.deepcopy(model).to(DEV), C, DEV, args, compute_dtype=None)
        assert eng.sequential and eng.tf is None
        eng.use_graphs = graphs
        eng.load_global(eng.layout.flatten(model.state_dict(), device=DEV))
        losses = []
        for t in tables:
            eng.class_weight = t.to(DEV)          # a fresh tensor each round, as ValuedRCCLSimulator.run_round does
            losses.append(float(eng.train(store, torch.arange(C, device=DEV), 1, 32, 1e-3, shuffle=False)))
        torch.cuda.synchronize()
        outs.append((losses, eng.params.clone()))
        eng.close()
    (l0, p0), (l1, p1) = outs
    init = ParamLayout.from_module(model).flatten(model.state_dict(), device=DEV)
    for a, b in zip(l0, l1):
        assert abs(a - b) / abs(a) < 1e-3, (l0, l1)
    assert float((p0 - p1).norm() / (p0 - init).norm()) < 1e-3
