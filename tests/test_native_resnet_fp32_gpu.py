"""fp32 (reference-precision) native ResNet path: every conv/BN kernel's ``_f32`` instance against a
plain PyTorch fp32 reference of the same op, the whole native step against per-client fp32 torch,
and a multi-round FedAvg loss curve of the RCCL simulator on a ResNet-56-shaped config against the
reference's training loop (per-client deepcopy + SGD + weighted state_dict average,
``simulation/single_process/fedavg/fedavg_api.py:83-141``, ``my_model_trainer_classification.py:18-93``)."""
import copy

import pytest
import torch

from fedml_amd.core.arena import ParamLayout
from fedml_amd.models.cv.resnet import BasicBlock, Bottleneck, ResNet, resnet56
from fedml_amd.parallel.native_resnet import NativeResNetStep

pytestmark = pytest.mark.gpu
DEV = "cuda"
F32 = torch.float32


# Every test runs under both fp32 matrix-core modes (csrc/prec.h): exact v_mfma_f32_16x16x4_f32 products,
# and the split-bf16 mode (three bf16 MFMAs per fragment, ~2^-16 relative per product). Kernel checks
# stated as "< 1e-5" hold at 1e-5 for exact and at 1e-4 for bf16x3 (TOL scales every relative error).
# The whole-step check derives its bound from measured spreads at the mode's product precision (see
# test_native_step_f32_matches_reference). The 10-round loss curve is bounded by the CPU-vs-GPU PyTorch
# fp32 spread; split-bf16 products (~2^-16) drift further from it than exact fp32 — measured: 10-round
# deviation 1.11e-2 against an exact-mode bound of 9.4e-3 (3 x the 3.1e-3 spread), i.e. 1.18x — so that
# one bound is 3x under bf16x3 (bf16 storage sits at 2-4e-1 on the same checks).
TOL = {"exact": 1.0, "bf16x3": 10.0}
STEP_TOL = {"exact": 1.0, "bf16x3": 3.0}
_mode = ["exact"]


@pytest.fixture(autouse=True, params=["exact", "bf16x3"])
def f32_mma(request):
    from fedml_amd.ops import nn_ops
    _mode[0] = request.param
    nn_ops.set_f32_mma_mode(request.param)
    yield request.param
    nn_ops.set_f32_mma_mode("exact")
    _mode[0] = "exact"


def rel(a, b):
    err = float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))
    return err / TOL[_mode[0]]


@pytest.mark.parametrize("ch,hw,stride", [(16, 32, 1), (32, 16, 1), (64, 8, 1), (32, 32, 2), (64, 16, 2), (32, 16, 2),
                                         (16, 16, 1)])
@pytest.mark.parametrize("N", [8, 16])
def test_conv3x3_f32_kernels(ch, hw, stride, N):
    from fedml_amd.ops import nn_ops
    torch.manual_seed(0)
    C = 3
    K = 9 * ch
    ldk = (K + 31) // 32 * 32 + 8
    x = torch.randn(C, N, hw, hw, ch, device=DEV)
    wpk = torch.zeros(C, ch, ldk, device=DEV)
    wpk[:, :, :K] = torch.randn(C, ch, K, device=DEV) * 0.1
    s = torch.rand(C, ch, device=DEV) + 0.5
    t = torch.randn(C, ch, device=DEV) * 0.1
    wt = wpk[:, :, :K].view(C, ch, 3, 3, ch).permute(0, 1, 4, 2, 3)
    wt_b = wpk[:, :, :K].view(C, ch, 3, 3, ch).permute(0, 4, 1, 2, 3)
    ho = hw // stride
    y3 = torch.zeros(C, N, ho, ho, ch, device=DEV)
    st3 = torch.zeros(C, ch, 2, device=DEV)
    nn_ops.conv3x3_fwd(x, wpk, ch * ldk, s, t, y3, st3, C, N, hw, hw, ch, ch, ldk, stride)
    torch.cuda.synchronize()
    for c in range(C):
        xa = torch.relu(x[c] * s[c] + t[c]).permute(0, 3, 1, 2)
        ref = torch.nn.functional.conv2d(xa, wt[c], padding=1, stride=stride).permute(0, 2, 3, 1)
        assert rel(y3[c], ref) < 1e-5
        assert rel(st3[c, :, 0], ref.sum((0, 1, 2))) < 1e-4
        assert rel(st3[c, :, 1], (ref * ref).sum((0, 1, 2))) < 1e-5
    g = torch.randn(C, N, ho, ho, ch, device=DEV)
    yv = torch.randn(C, N, ho, ho, ch, device=DEV)
    al, be = torch.rand(C, ch, device=DEV), torch.randn(C, ch, device=DEV) * 0.1
    ga = torch.randn(C, ch, device=DEV) * 0.01
    ex = torch.randn(C, N, hw, hw, ch, device=DEV)
    dx = torch.zeros_like(ex)
    st = torch.zeros(C, ch, 3, device=DEV)
    nn_ops.conv3x3_bwd_data(g, yv, al, be, ga, wpk, ch * ldk, dx, ex, s, t, st, C, N, hw, hw, ch, ch, ldk, stride)
    torch.cuda.synchronize()
    for c in range(C):
        dy = (al[c] * g[c] + be[c] * yv[c] + ga[c]).permute(0, 3, 1, 2)
        ref = torch.nn.grad.conv2d_input((N, ch, hw, hw), wt_b[c], dy, padding=1, stride=stride).permute(0, 2, 3, 1)
        ref = ref * ((ex[c] * s[c] + t[c]) > 0)
        assert rel(dx[c], ref) < 1e-5
        assert rel(st[c, :, 0], ref.sum((0, 1, 2))) < 1e-4
        assert rel(st[c, :, 1], (ref * ex[c]).sum((0, 1, 2))) < 1e-4
    P = ch * ch * 9 + 64
    garena = torch.zeros(C, P, device=DEV)
    scratch = torch.zeros(C * ch * K, device=DEV)
    nn_ops.conv3x3_wgrad(g, yv, al, be, ga, x, s, t, garena, 16, C, N, hw, hw, ch, ch, ch, scratch, stride)
    torch.cuda.synchronize()
    for c in range(C):
        dy = (al[c] * g[c] + be[c] * yv[c] + ga[c]).permute(0, 3, 1, 2)
        xa = torch.relu(x[c] * s[c] + t[c]).permute(0, 3, 1, 2)
        ref = torch.nn.grad.conv2d_weight(xa, (ch, ch, 3, 3), dy, padding=1, stride=stride)
        assert rel(garena[c, 16:16 + ch * ch * 9], ref.reshape(-1)) < 1e-5


@pytest.mark.parametrize("cin,cout,epi", [(16, 64, 2), (32, 128, 2), (64, 256, 2), (64, 16, 3), (128, 32, 3),
                                          (256, 64, 3), (16, 16, 3), (64, 32, 3), (128, 64, 3)])
@pytest.mark.parametrize("M,ppw", [(8 * 16 * 16, 512), (5 * 7 * 7, 64), (1024, 256), (4096, 512), (16384, 512)])
def test_conv1x1_bwd_fused_f32(cin, cout, epi, M, ppw):
    from fedml_amd.ops import nn_ops
    torch.manual_seed(2)
    C = 3
    g = torch.randn(C, M, cout, device=DEV)
    yv = torch.randn(C, M, cout, device=DEV)
    al, be = torch.rand(C, cout, device=DEV), torch.randn(C, cout, device=DEV) * 0.1
    ga = torch.randn(C, cout, device=DEV) * 0.01
    W = torch.randn(C, cout, cin, device=DEV) / cin ** 0.5
    ld = (cout + 31) // 32 * 32 + 8
    wb = torch.zeros(C, cin * ld + 64, device=DEV)
    wb[:, :cin * ld].view(C, cin, ld)[:, :, :cout] = W.transpose(1, 2)
    e_x = torch.randn(C, M, cin, device=DEV)
    s = t = e_add = e_y1 = e_y2 = None
    if epi == 2:
        s, t = torch.rand(C, cin, device=DEV) + 0.5, torch.randn(C, cin, device=DEV) * 0.1
    else:
        e_add, e_y1, e_y2 = (torch.randn(C, M, cin, device=DEV) for _ in range(3))
    out = torch.empty(C, M, cin, device=DEV)
    stats = torch.zeros(C, cin, 3, device=DEV)
    garena = torch.zeros(C, cin * cout + 48, device=DEV)
    nn_ops.conv1x1_bwd_fused(g, yv, al, be, ga, wb, wb.stride(0), ld, e_x, s, t, e_add, e_y1, e_y2, out, stats,
                             garena, 16, C, M, cin, cout, epi, ppw)
    torch.cuda.synchronize()
    for c in range(C):
        dy = al[c] * g[c] + be[c] * yv[c] + ga[c]
        dx = dy @ W[c]
        xr = e_x[c]
        if epi == 2:
            gp = torch.where(xr * s[c] + t[c] > 0, dx, torch.zeros_like(dx))
            st = torch.stack([gp.sum(0), (gp * xr).sum(0)], -1)
            act = torch.relu(xr * s[c] + t[c])
        else:
            gp = torch.where(xr > 0, dx + e_add[c], torch.zeros_like(dx))
            st = torch.stack([gp.sum(0), (gp * e_y1[c]).sum(0), (gp * e_y2[c]).sum(0)], -1)
            act = xr
        assert rel(out[c], gp) < 1e-5
        assert rel(stats[c, :, :st.shape[-1]], st) < 1e-4
        assert rel(garena[c, 16:16 + cin * cout].view(cout, cin), dy.t() @ act) < 1e-5


@pytest.mark.parametrize("cin,cout,hw", [(16, 64, 32), (64, 16, 32), (32, 128, 16), (256, 64, 8), (64, 256, 8)])
def test_conv1x1_wgrad_f32(cin, cout, hw):
    from fedml_amd.ops import nn_ops
    torch.manual_seed(1)
    C, N = 3, 8
    x = torch.randn(C, N, hw, hw, cin, device=DEV)
    g = torch.randn(C, N, hw, hw, cout, device=DEV)
    yv = torch.randn(C, N, hw, hw, cout, device=DEV)
    al, be = torch.rand(C, cout, device=DEV), torch.randn(C, cout, device=DEV) * 0.1
    ga = torch.randn(C, cout, device=DEV) * 0.01
    s, t = torch.rand(C, cin, device=DEV) + 0.5, torch.randn(C, cin, device=DEV) * 0.1
    garena = torch.zeros(C, cin * cout + 48, device=DEV)
    nn_ops.conv1x1_wgrad(g, yv, al, be, ga, x, s, t, garena, 16, C, N * hw * hw, cin, cout, 512)
    torch.cuda.synchronize()
    for c in range(C):
        dy = (al[c] * g[c] + be[c] * yv[c] + ga[c]).reshape(-1, cout)
        xa = torch.relu(x[c] * s[c] + t[c]).reshape(-1, cin)
        assert rel(garena[c, 16:16 + cin * cout].view(cout, cin), dy.t() @ xa) < 1e-5


@pytest.mark.parametrize("cin,cout,k,stride,hw", [(8, 16, 3, 1, 32), (64, 128, 1, 2, 16), (128, 256, 1, 2, 8),
                                                   (16, 64, 1, 1, 16)])
def test_generic_conv_f32_kernels(cin, cout, k, stride, hw):
    """Implicit-GEMM forward / backward-data / weight-gradient kernels (stem and strided shortcut)."""
    from fedml_amd.ops import nn_ops
    torch.manual_seed(3)
    C, N = 2, 8
    pad = k // 2
    ho = (hw + 2 * pad - k) // stride + 1
    K = k * k * cin
    ldk = (K + 31) // 32 * 32 + 8
    K2 = k * k * cout
    ldk2 = (K2 + 31) // 32 * 32 + 8
    w = torch.randn(C, cout, cin, k, k, device=DEV) * 0.1
    wf = torch.zeros(C, cout, ldk, device=DEV)
    wf[:, :, :K] = w.permute(0, 1, 3, 4, 2).reshape(C, cout, K)
    wb = torch.zeros(C, cin, ldk2, device=DEV)
    wb[:, :, :K2] = w.permute(0, 2, 3, 4, 1).reshape(C, cin, K2)
    x = torch.randn(C, N, hw, hw, cin, device=DEV)
    y = torch.zeros(C, N, ho, ho, cout, device=DEV)
    st = torch.zeros(C, cout, 2, device=DEV)
    nn_ops.conv_fwd(x, wf, cout * ldk, None, None, y, st, C, N, hw, hw, cin, cout, k, k, stride, pad, ho, ho, ldk, 1)
    g = torch.randn(C, N, ho, ho, cout, device=DEV)
    yv = torch.randn(C, N, ho, ho, cout, device=DEV)
    al, be = torch.rand(C, cout, device=DEV), torch.randn(C, cout, device=DEV) * 0.1
    ga = torch.randn(C, cout, device=DEV) * 0.01
    dx = torch.zeros(C, N, hw, hw, cin, device=DEV)
    st_b = torch.zeros(C, cin, 3, device=DEV)
    data_grad = cin % 16 == 0          # the stem (3 → 8 padded input channels) needs no input gradient
    if data_grad:
        nn_ops.conv_bwd_data(g, yv, al, be, ga, wb, cin * ldk2, dx, nn_ops.EPI_STORE, None, None, None, None, None,
                             None, st_b, C, N, ho, ho, cout, cin, k, k, stride, pad, hw, hw, ldk2, 1)
    P = cout * cin * k * k + 32
    garena = torch.zeros(C, P, device=DEV)
    scratch = torch.zeros(C * cout * K, device=DEV)
    nn_ops.conv_wgrad(g, yv, al, be, ga, x, None, None, garena, 16, C, N, hw, hw, cin, ho, ho, cout, k, k, stride,
                      pad, 256, cin, scratch)
    torch.cuda.synchronize()
    for c in range(C):
        xc = x[c].permute(0, 3, 1, 2)
        ref = torch.nn.functional.conv2d(xc, w[c], stride=stride, padding=pad)
        assert rel(y[c].permute(0, 3, 1, 2), ref) < 1e-5
        dy = (al[c] * g[c] + be[c] * yv[c] + ga[c]).permute(0, 3, 1, 2)
        if data_grad:
            rdx = torch.nn.grad.conv2d_input(xc.shape, w[c], dy, stride=stride, padding=pad)
            assert rel(dx[c].permute(0, 3, 1, 2), rdx) < 1e-5
        rdw = torch.nn.grad.conv2d_weight(xc, w[c].shape, dy, stride=stride, padding=pad)
        assert rel(garena[c, 16:16 + cout * cin * k * k].view_as(rdw), rdw) < 1e-5


def _native_masks(step, c):
    """The ReLU masks client ``c``'s native forward used, NCHW bool, in network order: stem, then per block its
    inner activations relu(y_j·s_j + t_j) (evaluated in fp64 — the product of two fp32 values and its sum with
    a third keep their sign exactly) and its stored block output (> 0)."""
    def inner(y, v):
        return (y[c].double() * v[0, c].double() + v[1, c].double() > 0).permute(0, 3, 1, 2)
    masks = [(step.stem_out[c] > 0).permute(0, 3, 1, 2)]
    for b in step.blocks:
        assert all(y is not None for y in b.ys), "recomputed-y blocks keep no activation to read the mask from"
        for j in range(len(b.convs) - 1):
            masks.append(inner(b.ys[j], step.bn_vec[b.bns[j].key]))
        masks.append((b.out[c] > 0).permute(0, 3, 1, 2))
    return masks


def _masked_fp64_grads(step, layout, flat, x, y, masks):
    """One client's fp64 step through the native step's own layer specs, every ReLU replaced by the given mask
    (``masks`` in ``_native_masks`` order, None → the fp64 sign itself). Returns (loss, {key: grad}, flips):
    flips = mask positions where the given mask disagrees with the fp64 pre-activation's sign."""
    F = torch.nn.functional
    sd = layout.unflatten(flat.double().cpu())
    prm = {s.key: sd[s.key].double().requires_grad_(True) for s in layout.slots if s.trainable}
    it = iter(masks) if masks is not None else None
    flips = [0]

    def relu(z):
        if it is None:
            return torch.relu(z)
        m = next(it).cpu()
        flips[0] += int(((z.detach() > 0) != m).sum())
        return z * m.to(z.dtype)

    def conv(cv, h):
        return F.conv2d(h, prm[cv.key], stride=cv.stride, padding=cv.pad)

    def bn(spec, h):
        return F.batch_norm(h, None, None, prm[f"{spec.key}.weight"], prm[f"{spec.key}.bias"], True, 0.0, spec.eps)

    h = relu(bn(step.stem[1], conv(step.stem[0], x.double())))
    for b in step.blocks:
        z = h
        for j, (cv, sp) in enumerate(zip(b.convs, b.bns)):
            z = bn(sp, conv(cv, z))
            if j < len(b.convs) - 1:
                z = relu(z)
        sc = bn(b.ds_bn, conv(b.ds_conv, h)) if b.ds_conv is not None else h
        h = relu(z + sc)
    logits = F.linear(h.mean((2, 3)), prm["fc.weight"], prm["fc.bias"])
    loss = F.cross_entropy(logits, y.cpu())
    loss.backward()
    return float(loss.detach()), {k: p.grad for k, p in prm.items()}, flips[0]


@pytest.mark.parametrize("builder,hw", [
    (lambda: ResNet(Bottleneck, [1, 1, 1], 10), 16),
    (lambda: ResNet(BasicBlock, [2, 1, 1], 10), 16),
    (lambda: ResNet(Bottleneck, [2, 2, 2], 100), 32),
])
@pytest.mark.parametrize("det", [False, True], ids=["fp32_atomics", "deterministic"])
def test_native_step_f32_matches_reference(builder, hw, det):
    """The fp32 native step against an fp64 step that uses the native step's OWN ReLU masks — in the production
    configuration (fp32 atomics, deferred BN finalisation folded into the consumer kernels) and in
    deterministic mode (fixed-point cross-workgroup sums, explicit BN finalisation).

    A ReLU pre-activation within rounding of 0 makes its mask — and every upstream gradient — depend on the
    last bits of the BN scale/shift: one such flip moves gradients of these random-init nets by 1e-4..1e-2
    for ANY fp32 implementation (round 3: the driver's box saw native median 2.6e-3 vs fp64 on
    ``Bottleneck,[2,2,2]``). Reading the masks back from the native activations (stored pre-BN outputs and
    BN scale/shift, block outputs) and forcing them on the fp64 step removes that discontinuity, so the
    comparison is a plain fp32-vs-fp64 rounding bound on every slot. The number of masks the native step
    set differently from fp64's own signs is reported and must stay a vanishing fraction (only elements
    at the threshold can flip); a kernel bug shows up as a large per-slot error, not as flips."""
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
    step = NativeResNetStep(model, layout, C, DEV, dtype=F32)
    if det:
        step.enable_deterministic()
    assert step._lazy_on() == (not det)
    try:
        assert step.dtype == F32
        loss = float(step.step(arena, garena, x, y, row_scale, active))
        torch.cuda.synchronize()
        assert step.packed.dtype == F32 and step.x_in.dtype == F32
        ref_loss, worst, flips, n_mask, errs = 0.0, 0.0, 0, 0, []
        for c in range(C):
            masks = _native_masks(step, c)
            n_mask += sum(int(m.numel()) for m in masks)
            lc, gref, fl = _masked_fp64_grads(step, layout, flat, x[c].cpu(), y[c], masks)
            ref_loss += lc
            flips += fl
            for s in layout.slots:
                if s.key not in gref:
                    continue
                r = gref[s.key].reshape(-1)
                e = float((garena[c, s.offset:s.offset + s.numel].double().cpu() - r).norm()
                          / r.norm().clamp_min(1e-30))
                errs.append((e, c, s.key))
    finally:
        step.close()
    errs.sort(reverse=True)
    med = errs[len(errs) // 2][0]
    print(f"[{_mode[0]}] masked-fp64 slot error max {errs[0][0]:.2e} ({errs[0][2]}) median {med:.2e}; "
          f"native masks differing from fp64 signs: {flips} of {n_mask}")
    assert abs(loss - ref_loss) / ref_loss < 1e-5 * TOL[_mode[0]], (loss, ref_loss)
    assert flips <= max(8, n_mask // 100000), (flips, n_mask)
    # fp32 storage, fp32 accumulation: per-slot relative error a few fp32 ulps times the depth's growth
    assert errs[0][0] < 1e-4 * TOL[_mode[0]], errs[:8]
    assert med < 1e-5 * TOL[_mode[0]], med
    s = layout.slot("bn1.running_mean")
    m = copy.deepcopy(model).to(DEV)
    m.train()
    m(x[0])
    assert torch.allclose(arena[0, s.offset:s.offset + s.numel], m.bn1.running_mean, atol=1e-5, rtol=1e-4)


def _reference_fedavg(model, x, y, K, n, bs, lr, rounds, device=DEV):
    """The reference's SP FedAvg round, fp32: clients one after another on a deepcopy of the global
    state, SGD without momentum / weight decay, per-batch loss, sample-weighted state_dict average
    (all entries, BN buffers included)."""
    x, y = x.to(device), y.to(device)
    glob = copy.deepcopy(model).to(device).float().state_dict()
    losses = []
    for _ in range(rounds):
        states, round_loss, nb = [], 0.0, 0
        for c in range(K):
            m = copy.deepcopy(model).to(device).float()
            m.load_state_dict(glob)
            m.train()
            opt = torch.optim.SGD(m.parameters(), lr=lr)
            for lo in range(0, n, bs):
                xb, yb = x[c * n + lo:c * n + lo + bs], y[c * n + lo:c * n + lo + bs]
                m.zero_grad()
                loss = torch.nn.functional.cross_entropy(m(xb), yb)
                loss.backward()
                opt.step()
                round_loss += float(loss)
                nb += 1
            states.append(m.state_dict())
        glob = {k: sum(st[k].float() for st in states) / K for k in glob}
        losses.append(round_loss / nb)
    return losses


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_fedavg_resnet56_loss_curve_tracks_fp32_torch(dtype, f32_mma):
    """10 FedAvg rounds of ResNet-56 / CIFAR-100-shaped synthetic data through the RCCL simulator (native
    HIP step, HIP graphs, on-GPU aggregation) against the reference's fp32 training loop run by PyTorch on
    the GPU. Training amplifies last-bit differences (ReLU masks at the threshold, see above), so the
    yardstick is the spread between two valid fp32 implementations — the same loop in PyTorch on the CPU
    vs on the GPU: native fp32 must stay within 3× that spread (floor 0.5 %), native bf16 within 5 %;
    both must learn."""
    from fedml_amd.arguments import Arguments
    from fedml_amd.data.synthetic import get_spec
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.simulator import RCCLSimulator
    if dtype == "bf16" and f32_mma != "exact":
        pytest.skip("the fp32 matrix-core mode does not apply to bf16 storage")
    torch.manual_seed(0)
    K, n, bs, lr, rounds = 4, 64, 32, 0.02, 10
    spec = get_spec("cifar100")
    store = DeviceClientStore.synthetic_on_device(spec, [n] * K, torch.device(DEV), seed=0)
    model = resnet56(100)
    ref = _reference_fedavg(model, store.x_all, store.y_all, K, n, bs, lr, rounds)
    args = Arguments.from_dict({"x": {
        "training_type": "simulation", "backend": "RCCL", "federated_optimizer": "FedAvg", "dataset": "cifar100",
        "model": "resnet56", "client_num_in_total": K, "client_num_per_round": K, "comm_round": rounds,
        "epochs": 1, "batch_size": bs, "client_optimizer": "sgd", "learning_rate": lr, "shuffle": False,
        "frequency_of_the_test": 0, "compute_dtype": dtype, "random_seed": 0, "fp32_mma": f32_mma}})
    sim = RCCLSimulator(args, torch.device(DEV), None, copy.deepcopy(model), store=store)
    assert sim.engine.native_step is not None
    assert sim.engine.native_step.dtype == (F32 if dtype == "fp32" else torch.bfloat16)
    sim.run(rounds)
    got = [sim.history[r]["train_loss"] for r in range(rounds)]
    sim.close()
    dev = max(abs(a - b) / b for a, b in zip(got, ref))
    if dtype == "fp32":
        cpu = _reference_fedavg(model, store.x_all, store.y_all, K, n, bs, lr, rounds, device="cpu")
        spread = max(abs(a - b) / b for a, b in zip(cpu, ref))
        assert dev < max(3 * spread, 5e-3) * STEP_TOL[f32_mma], (dev, spread, list(zip(got, ref, cpu)))
    else:
        assert dev < 0.05, (dev, list(zip(got, ref)))
    assert got[-1] < got[0] - 0.1      # it learns


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 5e-3), (torch.bfloat16, 0.5)])
def test_native_step_heterogeneous_counts(dtype, tol):
    """Clients with different batch sizes in ONE native step (nimg = [16, 11, 3, 0]): every client's
    gradients equal its own fp64 PyTorch step on its valid samples; BatchNorm normalises over them only;
    the empty client gets exactly zero gradients and unchanged BN running statistics."""
    torch.manual_seed(0)
    model = ResNet(Bottleneck, [1, 1, 1], 10)
    layout = ParamLayout.from_module(model)
    C, N, hw = 4, 16, 16
    counts = [16, 11, 3, 0]
    flat = layout.flatten(model.state_dict()).to(DEV)
    arena = flat.view(1, -1).repeat(C, 1).contiguous()
    garena = torch.zeros_like(arena)
    x = torch.randn(C, N, 3, hw, hw, device=DEV)
    y = torch.randint(0, 10, (C, N), device=DEV)
    mask = torch.arange(N, device=DEV).view(1, -1) < torch.tensor(counts, device=DEV).view(-1, 1)
    row_scale = mask.float() / torch.tensor([max(1, b) for b in counts], device=DEV).view(-1, 1)
    active = torch.tensor([1.0 if b else 0.0 for b in counts], device=DEV)
    nimg = torch.tensor(counts, dtype=torch.int32, device=DEV)
    step = NativeResNetStep(model, layout, C, DEV, dtype=dtype)
    loss = float(step.step(arena, garena, x, y, row_scale, active, nimg=nimg))
    torch.cuda.synchronize()
    ref_loss = 0.0
    for c, b in enumerate(counts):
        g = garena[c]
        if b == 0:
            assert float(g.abs().max()) == 0.0
            assert torch.equal(arena[c], flat)          # running statistics untouched
            continue
        m = copy.deepcopy(model).double()
        m.load_state_dict({k: v.double() if v.is_floating_point() else v
                           for k, v in layout.unflatten(flat.cpu()).items()})
        m.train()
        lo = torch.nn.functional.cross_entropy(m(x[c, :b].cpu().double()), y[c, :b].cpu())
        lo.backward()
        ref_loss += float(lo)
        sd = {k: p.grad for k, p in m.named_parameters()}
        for s in layout.slots:
            if s.key in sd:
                r = sd[s.key].reshape(-1)
                err = float((g[s.offset:s.offset + s.numel].cpu().double() - r).norm() / r.norm().clamp_min(1e-30))
                assert err < tol * (STEP_TOL[_mode[0]] if dtype == torch.float32 else 1.0), (c, s.key, err)
        rm = layout.slot("bn1.running_mean")
        assert torch.allclose(arena[c, rm.offset:rm.offset + rm.numel].cpu().double(),
                              m.bn1.running_mean, rtol=1e-3 if dtype == torch.float32 else 5e-2, atol=1e-4)
    assert abs(loss - ref_loss) / ref_loss < (1e-5 * TOL[_mode[0]] if dtype == torch.float32 else 2e-2)


def test_engine_heterogeneous_partition_stays_native():
    """A Dirichlet-like partition (clients of 150, 97, 20 and 0 samples, batch 32): the engine keeps every
    step on the captured native program (no torch interpreter fallback) and one local epoch equals each
    client's own fp32 PyTorch SGD epoch (reference trainer semantics: my_model_trainer_classification.py)."""
    from fedml_amd.arguments import Arguments
    from fedml_amd.simulation.rccl.client_store import DeviceClientStore
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    torch.manual_seed(0)
    model = ResNet(Bottleneck, [1, 1, 1], 10)
    counts = [150, 97, 20, 0]
    n = sum(counts)
    offs = [0, 150, 247, 267]
    store = DeviceClientStore(torch.randn(n, 3, 16, 16, device=DEV), torch.randint(0, 10, (n,), device=DEV),
                              offs, counts)
    lr, bs = 0.02, 32
    args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": lr}})
    eng = ClientBatchEngine(copy.deepcopy(model).to(DEV), 4, DEV, args, compute_dtype=None)
    assert eng.native_step is not None and eng.native_step.dtype == F32
    flat = eng.layout.flatten(model.state_dict(), device=DEV)
    eng.load_global(flat)
    calls = []
    orig = eng._step_loss
    eng._step_loss = lambda *a, **k: calls.append(1) or orig(*a, **k)
    eng.train(store, torch.arange(4, device=DEV), 1, bs, lr, shuffle=False)
    torch.cuda.synchronize()
    assert not calls and len(eng._graphs) >= 2       # every step replayed a native graph
    for c, cnt in enumerate(counts):
        if cnt == 0:
            assert torch.equal(eng.params[c], flat)
            continue
        m = copy.deepcopy(model).to(DEV)
        m.train()
        opt = torch.optim.SGD(m.parameters(), lr=lr)
        for lo in range(0, cnt, bs):
            xb = store.x_all[offs[c] + lo:offs[c] + min(cnt, lo + bs)]
            yb = store.y_all[offs[c] + lo:offs[c] + min(cnt, lo + bs)]
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(xb), yb).backward()
            opt.step()
        ref = eng.layout.flatten(m.state_dict(), device=DEV)
        upd_ref = ref - flat
        err = float((eng.params[c] - ref).norm() / upd_ref.norm())
        assert err < 2e-2, (c, err)
    eng.close()
