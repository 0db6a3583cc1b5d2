"""Round-4 diagnostics (GPU): (1) MobileNet batched interpreter, native plane/bconv kernels vs PyTorch ops, per
parameter gradient of one step; (2) native ResNet step: padded batch geometry (N=8, nimg=5) vs exact (N=5), and
deferred vs explicit BN finalisation."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def mobilenet_grads():
    from fedml_amd.core.arena import ParamLayout
    from fedml_amd.models.cv.mobilenet import mobilenet
    from fedml_amd.parallel import batched_nn
    torch.manual_seed(0)
    model = mobilenet(10).cuda()
    C, B = 2, 16
    layout = ParamLayout.from_module(model)
    x = torch.randn(C, B, 3, 32, 32, device="cuda")
    y = torch.randint(0, 10, (C, B), device="cuda")

    def run(native):
        batched_nn._NATIVE_BCONV = native
        params = layout.alloc_stack(C, "cuda")
        grads = layout.alloc_stack(C, "cuda")
        flat = layout.flatten(model.state_dict(), device="cuda")
        params.copy_(flat.view(1, -1).expand(C, -1))
        views = {}
        for s in layout.slots:
            v = params[:, s.offset:s.offset + s.numel].view(C, *s.shape)
            if s.trainable:
                v = v.detach().requires_grad_(True)
                v.grad = grads[:, s.offset:s.offset + s.numel].view(C, *s.shape)
            views[s.key] = v
        it = batched_nn.BatchedInterpreter(model, layout, C)
        out = it.run(views, x, training=True)
        loss = torch.nn.functional.cross_entropy(out.reshape(C * B, -1), y.reshape(-1))
        loss.backward()
        it.flush_deferred()
        torch.cuda.synchronize()
        return out.detach(), grads.clone(), params.clone()

    o1, g1, p1 = run(True)
    o0, g0, p0 = run(False)
    print("mobilenet logits rel", rel(o1, o0))
    worst = []
    for s in layout.slots:
        a, b = g1[:, s.offset:s.offset + s.numel], g0[:, s.offset:s.offset + s.numel]
        if s.trainable and float(b.norm()) > 0:
            worst.append((rel(a, b), s.key))
        else:
            e = rel(p1[:, s.offset:s.offset + s.numel], p0[:, s.offset:s.offset + s.numel])
            if e > 1e-5:
                worst.append((e, s.key + " (buffer)"))
    worst.sort(reverse=True)
    for e, k in worst[:12]:
        print(f"  grad rel {e:.3e}  {k}")


def resnet_geometry():
    from fedml_amd.core.arena import ParamLayout
    from fedml_amd.models.cv.resnet import Bottleneck, ResNet
    from fedml_amd.parallel.native_resnet import NativeResNetStep
    torch.manual_seed(0)
    model = ResNet(Bottleneck, [1, 1, 1], 10)
    layout = ParamLayout.from_module(model)
    C = 3
    flat = layout.flatten(model.state_dict()).cuda()
    xs = torch.randn(C, 8, 3, 16, 16, device="cuda")
    ys = torch.randint(0, 10, (C, 8), device="cuda")

    def run(N, nv, lazy, det=False):
        step = NativeResNetStep(model, layout, C, "cuda")
        step.use_lazy = lazy
        if det:
            step.enable_deterministic()
        arena = flat.view(1, -1).repeat(C, 1).contiguous()
        garena = torch.zeros_like(arena)
        x = xs[:, :N].contiguous()
        y = ys[:, :N].contiguous()
        rs = (torch.arange(N, device="cuda") < nv).float().view(1, -1).expand(C, N) / nv
        nimg = torch.full((C,), nv, dtype=torch.int32, device="cuda")
        loss = step.step(arena, garena, x, y, rs.contiguous(), torch.ones(C, device="cuda"), nimg=nimg)
        torch.cuda.synchronize()
        step.close()
        return float(loss), garena, arena

    _, gd1, ad1 = run(5, 5, True, det=True)
    _, gd0, ad0 = run(5, 5, False, det=True)
    print(f"resnet deterministic lazy-vs-explicit: grad bitwise {torch.equal(gd1, gd0)} arena bitwise "
          f"{torch.equal(ad1, ad0)} (rel {rel(gd1, gd0):.3e})")
    l5, g5, a5 = run(5, 5, True)
    l8, g8, a8 = run(8, 5, True)
    l5e, g5e, a5e = run(5, 5, False)
    print(f"resnet padded-vs-exact geometry: loss {l8:.7f} vs {l5:.7f}; grad rel {rel(g8, g5):.3e}; "
          f"arena rel {rel(a8 - flat, a5 - flat):.3e}")
    print(f"resnet lazy-vs-explicit: grad bitwise {torch.equal(g5, g5e)} rel {rel(g5, g5e):.3e}; arena bitwise "
          f"{torch.equal(a5, a5e)}")


if __name__ == "__main__":
    resnet_geometry()
