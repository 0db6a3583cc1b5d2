"""Round-4 diagnostic (GPU): deterministic mode with deferred BN finalisation vs deterministic explicit
finalisation, per parameter slot of one native ResNet step (which layer's gradient departs first)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def main():
    os.environ["FEDML_AMD_BN_LAZY_DET"] = "1"      # defer in deterministic mode too (the case under study)
    from fedml_amd.core.arena import ParamLayout
    from fedml_amd.models.cv.resnet import Bottleneck, ResNet
    from fedml_amd.parallel.native_resnet import NativeResNetStep
    torch.manual_seed(0)
    model = ResNet(Bottleneck, [1, 1, 1], 10)
    layout = ParamLayout.from_module(model)
    C, N = 3, 5
    flat = layout.flatten(model.state_dict()).cuda()
    xs = torch.randn(C, N, 3, 16, 16, device="cuda")
    ys = torch.randint(0, 10, (C, N), device="cuda")

    def run(lazy, det):
        step = NativeResNetStep(model, layout, C, "cuda")
        step.use_lazy = lazy
        if det:
            step.enable_deterministic()
        arena = flat.view(1, -1).repeat(C, 1).contiguous()
        garena = torch.zeros_like(arena)
        rs = torch.full((C, N), 1.0 / N, device="cuda")
        nimg = torch.full((C,), N, dtype=torch.int32, device="cuda")
        loss = step.step(arena, garena, xs, ys, rs, torch.ones(C, device="cuda"), nimg=nimg)
        torch.cuda.synchronize()
        step.close()
        return float(loss), garena.clone(), arena.clone()

    runs = {k: run(*k) for k in [(False, False), (True, False), (False, True), (True, True)]}
    ref = runs[(False, False)]
    for k, (l, g, a) in runs.items():
        print(f"lazy={k[0]} det={k[1]}: loss {l:.7f} (ref {ref[0]:.7f}) grad rel {rel(g, ref[1]):.3e} "
              f"arena rel {rel(a - flat, ref[2] - flat):.3e}")
    g1, g0 = runs[(True, True)][1], runs[(False, True)][1]
    print("det lazy vs det explicit, per slot (layout order):")
    for s in layout.slots:
        a, b = g1[:, s.offset:s.offset + s.numel], g0[:, s.offset:s.offset + s.numel]
        if not s.trainable:
            continue
        e = rel(a, b)
        if e > 1e-6:
            ratio = float(a.double().norm() / b.double().norm().clamp_min(1e-30))
            print(f"  {s.key:40s} rel {e:.3e}  |lazy|/|explicit| {ratio:.4f}")


if __name__ == "__main__":
    main()
