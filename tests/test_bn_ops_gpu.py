"""Fused channels-last BatchNorm(+residual+ReLU) HIP kernels (``csrc/bnc_kernels.hip``) against the
plain PyTorch fp32 reference of the same op: output, dx, dγ, dβ, d(residual), running statistics."""
import pytest
import torch
import torch.nn as nn

from fedml_amd.ops import bn_ops

pytestmark = pytest.mark.gpu


def _ref(bn, x, res, relu):
    out = bn(x)
    if res is not None:
        out = out + res
    return torch.relu(out) if relu else out


@pytest.mark.parametrize("C,N,HW", [(64, 16, 32), (128, 8, 16), (256, 8, 8), (512, 16, 4), (8, 4, 5)])
@pytest.mark.parametrize("relu,residual", [(True, False), (True, True), (False, False), (False, True)])
def test_bnc_matches_fp32_reference(C, N, HW, relu, residual):
    torch.manual_seed(C + HW)
    dev = "cuda"
    bn = nn.BatchNorm2d(C).to(dev).train()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
        bn.running_mean.uniform_(-0.1, 0.1)
    ref = nn.BatchNorm2d(C).to(dev).train()
    ref.load_state_dict(bn.state_dict())

    x = (torch.randn(N, C, HW, HW, device=dev) * 2 + 0.3).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    r = torch.randn_like(x) if residual else None
    x.requires_grad_(True)
    if r is not None:
        r.requires_grad_(True)
    assert bn_ops._fast_ok(bn, x, r)
    y = bn_ops.batch_norm_act(bn, x, residual=r, relu=relu)
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    dy = torch.randn_like(y)
    y.backward(dy)

    xf = x.detach().float().requires_grad_(True)
    rf = r.detach().float().requires_grad_(True) if r is not None else None
    yf = _ref(ref, xf, rf, relu)
    yf.backward(dy.float())

    torch.testing.assert_close(y.float(), yf, atol=4e-2, rtol=2e-2)
    torch.testing.assert_close(x.grad.float(), xf.grad, atol=4e-2, rtol=4e-2)
    torch.testing.assert_close(bn.weight.grad, ref.weight.grad, atol=0.5, rtol=2e-2)
    torch.testing.assert_close(bn.bias.grad, ref.bias.grad, atol=0.5, rtol=2e-2)
    if r is not None:
        torch.testing.assert_close(r.grad.float(), rf.grad, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(bn.running_var, ref.running_var, atol=1e-3, rtol=1e-3)
    assert int(bn.num_batches_tracked) == int(ref.num_batches_tracked) == 1


def test_bnc_resnet18_no_worse_than_module_path(monkeypatch):
    """ResNet-18 forward/backward under bf16 autocast in channels-last: the fused path's weight gradients
    are as close to the fp32 model's as the module (MIOpen BN) path's are (relative L2 error per tensor)."""
    from fedml_amd.models.cv.resnet import resnet18_cifar
    torch.manual_seed(0)
    models = [resnet18_cifar(10).cuda().to(memory_format=torch.channels_last).train() for _ in range(3)]
    for m in models[1:]:
        m.load_state_dict(models[0].state_dict())
    x = torch.randn(32, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last)
    grads = []
    for model, on, amp in ((models[0], True, True), (models[1], False, True), (models[2], False, False)):
        monkeypatch.setattr(bn_ops, "_ENABLED", on)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            loss = model(x).float().logsumexp(-1).mean()
        loss.backward()
        grads.append([p.grad.float() for p in model.parameters()])
    for gf, gm, g32 in zip(*grads):
        ef = ((gf - g32).norm() / (g32.norm() + 1e-12)).item()
        em = ((gm - g32).norm() / (g32.norm() + 1e-12)).item()
        assert ef <= 1.5 * em + 2e-2, (ef, em)
    torch.testing.assert_close(models[0].layer4[1].bn2.running_var, models[2].layer4[1].bn2.running_var,
                               atol=1e-2, rtol=2e-2)


def test_bnc_large_mean_offset():
    """mean 50, std 0.5 (bf16 input): the shifted statistics sums keep the variance accurate — the
    E[x²] − mean² form loses it to cancellation."""
    torch.manual_seed(3)
    dev = "cuda"
    C = 64
    bn = nn.BatchNorm2d(C).to(dev).train()
    ref = nn.BatchNorm2d(C).to(dev).train()
    ref.load_state_dict(bn.state_dict())
    x = (torch.randn(16, C, 16, 16, device=dev) * 0.5 + 50.0).to(torch.bfloat16) \
        .contiguous(memory_format=torch.channels_last)
    y = bn_ops.batch_norm_act(bn, x, relu=False)
    yf = ref(x.float())
    torch.testing.assert_close(y.float(), yf, atol=5e-2, rtol=2e-2)
    torch.testing.assert_close(bn.running_var, ref.running_var, atol=1e-4, rtol=2e-3)
    torch.testing.assert_close(bn.running_mean, ref.running_mean, atol=1e-3, rtol=1e-4)


def test_bnc_backward_twice_with_retained_graph():
    """A second backward through a retained graph (gradient-penalty style ClientTrainers) gives the same
    gradients as the first: the atomic backward sums are zeroed per backward."""
    torch.manual_seed(4)
    dev = "cuda"
    bn = nn.BatchNorm2d(64).to(dev).train()
    x = torch.randn(8, 64, 8, 8, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = bn_ops.batch_norm_act(bn, x, relu=True)
    dy = torch.randn_like(y)
    gx1, gw1 = torch.autograd.grad(y, (x, bn.weight), dy, retain_graph=True)
    gx2, gw2 = torch.autograd.grad(y, (x, bn.weight), dy)
    torch.testing.assert_close(gx1, gx2)
    torch.testing.assert_close(gw1, gw2)
