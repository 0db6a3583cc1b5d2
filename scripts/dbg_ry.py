"""Debug: recomputed-y vs stored-y native step — per-block output and per-slot gradient differences."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedml_amd.core.arena import ParamLayout  # noqa: E402
from fedml_amd.models.cv.resnet import Bottleneck, ResNet  # noqa: E402
from fedml_amd.parallel.native_resnet import NativeResNetStep  # noqa: E402

DEV = "cuda"


def run(flag, model, layout, flat, x, y):
    os.environ["FEDML_AMD_RECOMPUTE_Y"] = flag
    C, N = x.shape[0], x.shape[1]
    arena = flat.view(1, -1).repeat(C, 1).contiguous()
    garena = torch.zeros_like(arena)
    rs = torch.full((C, N), 1.0 / N, device=DEV)
    step = NativeResNetStep(model, layout, C, DEV, dtype=torch.float32)
    if os.environ.get("DBG_DET", "1") == "1":
        step.enable_deterministic()
    loss = float(step.step(arena, garena, x, y, rs, torch.ones(C, device=DEV)))
    torch.cuda.synchronize()
    step.close()
    return loss, garena, [b.out.clone() for b in step.blocks], step


torch.manual_seed(0)
model = ResNet(Bottleneck, [1, 1, 1], 10)
layout = ParamLayout.from_module(model)
flat = layout.flatten(model.state_dict()).to(DEV)
x = torch.randn(3, 16, 3, 16, 16, device=DEV)
y = torch.randint(0, 10, (3, 16), device=DEV)
l0, g0, o0, s0 = run("0", model, layout, flat, x, y)
l1, g1, o1, s1 = run("1", model, layout, flat, x, y)
print("loss", l0, l1)
for i, (u, v) in enumerate(zip(o0, o1)):
    d = (u - v).abs()
    print(f"block {i} out: max|d| {float(d.max()):.3e} rel {float(d.norm() / u.norm()):.3e} "
          f"nonzero {int((d > 0).sum())}/{d.numel()} nan {bool(torch.isnan(v).any())}")
for s in layout.slots:
    if s.trainable:
        sl = slice(s.offset, s.offset + s.numel)
        r = g0[:, sl]
        print(f"{s.key:32s} {float((g1[:, sl] - r).norm() / r.norm().clamp_min(1e-30)):.3e}")
