"""Wide-channel native path (BASELINE config 2, ResNet-18/CIFAR-10): the K-streamed implicit-GEMM
kernel (``convk_gemm_kernel``, 128-512 channels, K up to 4608) and the output-channel-sliced weight
gradient against plain PyTorch fp32 references of the same ops, and the whole client-batched
ResNet-18 step against an fp64 per-client reference (``model/cv/resnet.py`` of the reference;
``simulation/single_process/fedavg/my_model_trainer_classification.py:18-93`` trains it in fp32)."""
import pytest
import torch

from fedml_amd.core.arena import ParamLayout
from fedml_amd.models.cv.resnet import ResNet18Cifar
from fedml_amd.parallel.native_resnet import NativeResNetStep

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


@pytest.fixture
def f32_mma(request):
    from fedml_amd.ops import nn_ops
    nn_ops.set_f32_mma_mode(request.param)
    yield request.param
    nn_ops.set_f32_mma_mode("exact")


# fp32 runs under both matrix-core modes (csrc/prec.h): exact fp32 products, and split-bf16 (bf16x3: ~2^-16
# per product, the K-streamed kernel stages pre-split hi/lo tiles) at 10x the exact tolerance
@pytest.mark.parametrize("dtype,tol,f32_mma", [(torch.float32, 2e-5, "exact"), (torch.float32, 2e-4, "bf16x3"),
                                               (torch.bfloat16, 2e-2, "exact")], indirect=["f32_mma"])
@pytest.mark.parametrize("cin,cout,k,stride,hw", [(128, 128, 3, 1, 16), (64, 128, 3, 2, 16), (256, 512, 3, 2, 8),
                                                   (512, 512, 3, 1, 4), (256, 512, 1, 2, 8), (128, 256, 3, 2, 16)])
def test_wide_conv_kernels(dtype, tol, f32_mma, cin, cout, k, stride, hw):
    """forward (BN+ReLU prologue, pivot, statistics), backward-data (folded BN backward operand, ReLU-mask
    epilogue + statistics) and weight gradient (128-channel dy slices for Cout > 256)."""
    from fedml_amd.ops import nn_ops
    torch.manual_seed(5)
    C, N = 2, 4
    pad = k // 2
    ho = (hw + 2 * pad - k) // stride + 1
    K, K2 = k * k * cin, k * k * cout
    ldk, ldk2 = (K + 31) // 32 * 32 + 8, (K2 + 31) // 32 * 32 + 8
    w = (torch.randn(C, cout, cin, k, k, device=DEV) * (2.0 / K) ** 0.5).to(dtype).float()
    wf = torch.zeros(C, cout, ldk, device=DEV, dtype=dtype)
    wf[:, :, :K] = w.permute(0, 1, 3, 4, 2).reshape(C, cout, K).to(dtype)
    wb = torch.zeros(C, cin, ldk2, device=DEV, dtype=dtype)
    wb[:, :, :K2] = w.permute(0, 2, 3, 4, 1).reshape(C, cin, K2).to(dtype)
    x = torch.randn(C, N, hw, hw, cin, device=DEV).to(dtype)
    s = (torch.rand(C, cin, device=DEV) + 0.5)
    t = torch.randn(C, cin, device=DEV) * 0.1
    piv = torch.randn(C, cout, device=DEV) * 0.1
    y = torch.zeros(C, N, ho, ho, cout, device=DEV, dtype=dtype)
    st = torch.zeros(C, cout, 2, device=DEV)
    nn_ops.conv_fwd(x, wf, cout * ldk, s, t, y, st, C, N, hw, hw, cin, cout, k, k, stride, pad, ho, ho, ldk, 1,
                    pivot=piv)
    g = torch.randn(C, N, ho, ho, cout, device=DEV).to(dtype)
    yv = torch.randn(C, N, ho, ho, cout, device=DEV).to(dtype)
    al, be = torch.rand(C, cout, device=DEV), torch.randn(C, cout, device=DEV) * 0.1
    ga = torch.randn(C, cout, device=DEV) * 0.01
    ex = torch.randn(C, N, hw, hw, cin, device=DEV).to(dtype)
    dx = torch.zeros(C, N, hw, hw, cin, device=DEV, dtype=dtype)
    st_b = torch.zeros(C, cin, 3, device=DEV)
    nn_ops.conv_bwd_data(g, yv, al, be, ga, wb, cin * ldk2, dx, nn_ops.EPI_MASK, ex, s, t, None, None, None, st_b, C,
                         N, ho, ho, cout, cin, k, k, stride, pad, hw, hw, ldk2, 1)
    P = cout * cin * k * k + 32
    garena = torch.zeros(C, P, device=DEV)
    scratch = torch.zeros(C * cout * K, device=DEV)
    nn_ops.conv_wgrad(g, yv, al, be, ga, x, s, t, garena, 16, C, N, hw, hw, cin, ho, ho, cout, k, k, stride, pad, 256,
                      cin, scratch)
    torch.cuda.synchronize()
    assert float(scratch.abs().max()) == 0.0   # scratch left zeroed for the next layer
    for c in range(C):
        xa = torch.relu(x[c].float() * s[c] + t[c]).permute(0, 3, 1, 2)
        ref = torch.nn.functional.conv2d(xa, w[c], stride=stride, padding=pad).permute(0, 2, 3, 1) - piv[c]
        assert rel(y[c], ref) < tol, ("fwd", rel(y[c], ref))
        assert rel(st[c, :, 0], y[c].float().sum((0, 1, 2))) < 1e-4
        assert rel(st[c, :, 1], (y[c].float() ** 2).sum((0, 1, 2))) < 1e-4
        dy = (al[c] * g[c].float() + be[c] * yv[c].float() + ga[c]).permute(0, 3, 1, 2)
        rdx = torch.nn.grad.conv2d_input((N, cin, hw, hw), w[c], dy, stride=stride, padding=pad).permute(0, 2, 3, 1)
        rdx = rdx * ((ex[c].float() * s[c] + t[c]) > 0)
        assert rel(dx[c], rdx) < tol, ("bwd", rel(dx[c], rdx))
        assert rel(st_b[c, :, 0], dx[c].float().sum((0, 1, 2))) < 1e-3
        assert rel(st_b[c, :, 1], (dx[c].float() * ex[c].float()).sum((0, 1, 2))) < 1e-3
        rdw = torch.nn.grad.conv2d_weight(xa, w[c].shape, dy, stride=stride, padding=pad)
        assert rel(garena[c, 16:16 + cout * cin * k * k].view_as(rdw), rdw) < tol, "wgrad"


def _ref_grads64(model, layout, flat, x, y, autocast=False):
    """fp64 per-client CPU gradients; ``autocast``: PyTorch's own bf16 mixed precision on the GPU instead."""
    import copy
    C = x.shape[0]
    grads = torch.zeros(C, layout.size, dtype=torch.float64)
    loss_sum = 0.0
    for c in range(C):
        m = copy.deepcopy(model).double() if not autocast else copy.deepcopy(model).to(DEV)
        m.load_state_dict({k: (v if not autocast else v.float().to(DEV)) for k, v in layout.unflatten(flat).items()})
        m.train()
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            out = m(x[c].double() if not autocast else x[c].to(DEV))
        loss = torch.nn.functional.cross_entropy(out.float() if autocast else out, y[c].to(out.device))
        loss.backward()
        loss_sum += float(loss)
        sd = {k: p.grad for k, p in m.named_parameters()}
        for sl in layout.slots:
            if sl.key in sd:
                grads[c, sl.offset:sl.offset + sl.numel] = sd[sl.key].reshape(-1).double().cpu()
    return loss_sum, grads


@pytest.mark.parametrize("dtype,f32_mma", [(torch.float32, "exact"), (torch.float32, "bf16x3"),
                                           (torch.bfloat16, "exact")], indirect=["f32_mma"])
def test_native_resnet18_step_matches_fp64(dtype, f32_mma):
    """The whole client-batched ResNet-18 step (every conv on the hand-written kernels) against an fp64
    per-client CPU reference: loss and every trainable slot's gradient. fp32: ≤ 1e-2 per slot (see
    test_native_step_f32_matches_reference for the ReLU-mask flips that set this bound). bf16: within
    2× (+0.05) of PyTorch's own bf16 autocast error on the same step (random-init ResNet-18 gradients
    through 18 bf16 layers are 0.2-0.4 off fp64 either way)."""
    torch.manual_seed(0)
    model = ResNet18Cifar(10)
    layout = ParamLayout.from_module(model)
    C, N = 2, 8
    flat = layout.flatten(model.state_dict()).to(DEV)
    arena = flat.view(1, -1).repeat(C, 1).contiguous()
    garena = torch.zeros_like(arena)
    x = torch.randn(C, N, 3, 32, 32, device=DEV)
    y = torch.randint(0, 10, (C, N), device=DEV)
    step = NativeResNetStep(model, layout, C, DEV, dtype=dtype)
    loss = float(step.step(arena, garena, x, y, torch.full((C, N), 1.0 / N, device=DEV), torch.ones(C, device=DEV)))
    torch.cuda.synchronize()
    ref_loss, ref = _ref_grads64(model, layout, flat.cpu().double(), x.cpu(), y.cpu())
    x3 = 10.0 if f32_mma == "bf16x3" else 1.0
    assert abs(loss - ref_loss) / ref_loss < (1e-5 * x3 if dtype == torch.float32 else 2e-2), (loss, ref_loss)
    amp = _ref_grads64(model, layout, flat.cpu().double(), x.cpu(), y.cpu(), autocast=True)[1] \
        if dtype == torch.bfloat16 else None
    bad = []
    for sl in layout.slots:
        if not sl.trainable:
            continue
        r = ref[:, sl.offset:sl.offset + sl.numel]
        err = rel(garena[:, sl.offset:sl.offset + sl.numel].cpu(), r)
        tol = 1e-2 * (3.0 if x3 > 1 else 1.0) if amp is None else 2 * rel(amp[:, sl.offset:sl.offset + sl.numel], r) + 0.05
        if err > tol:
            bad.append((sl.key, round(err, 5), round(tol, 5)))
    assert not bad, bad[:8]


def test_engine_runs_resnet18_natively():
    """The client-batched engine picks the native kernels for ResNet-18 at both precisions."""
    from fedml_amd.arguments import Arguments
    from fedml_amd.simulation.rccl.engine import ClientBatchEngine
    model = ResNet18Cifar(10).to(DEV)
    args = Arguments.from_dict({"x": {"client_optimizer": "sgd", "learning_rate": 0.01}})
    for cd in (None, torch.bfloat16):
        eng = ClientBatchEngine(model, 2, torch.device(DEV), args, compute_dtype=cd)
        assert eng.native_step is not None
