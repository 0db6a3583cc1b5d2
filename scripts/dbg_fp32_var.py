#!/usr/bin/env python3
"""Run-to-run spread of the fp32 native step (5 fresh runs, same inputs) and, per BN, the cancellation
ratio Σ|g| / |Σg| of its output gradient in an fp64 torch reference."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedml_amd.core.arena import ParamLayout  # noqa: E402
from fedml_amd.models.cv.resnet import Bottleneck, ResNet  # noqa: E402
from fedml_amd.parallel.native_resnet import NativeResNetStep  # noqa: E402

DEV = "cuda"
torch.manual_seed(0)
model = ResNet(Bottleneck, [1, 1, 1], 10)
layout = ParamLayout.from_module(model)
C, N, hw = 3, 16, 16
flat = layout.flatten(model.state_dict()).to(DEV)
x = torch.randn(C, N, 3, hw, hw, device=DEV)
y = torch.randint(0, 10, (C, N), device=DEV)
runs, stats = [], []
for r in range(5):
    arena = flat.view(1, -1).repeat(C, 1).contiguous()
    garena = torch.zeros_like(arena)
    st = NativeResNetStep(model, layout, C, DEV, dtype=torch.float32)
    st.step(arena, garena, x, y, torch.full((C, N), 1.0 / N, device=DEV), torch.ones(C, device=DEV))
    torch.cuda.synchronize()
    runs.append(garena.clone())
    stats.append({k: b.clone() for k, (f, b) in st.stat_views.items()})
sl = layout.slot("conv1.weight")
for r in range(1, 5):
    d = float((runs[r] - runs[0]).norm() / runs[0].norm())
    ds = float((runs[r][:, sl.offset:sl.offset + sl.numel] - runs[0][:, sl.offset:sl.offset + sl.numel]).norm()
               / runs[0][:, sl.offset:sl.offset + sl.numel].norm())
    print(f"run {r} vs 0: all {d:.2e} conv1.weight {ds:.2e}")
for k in stats[0]:
    sp = max(float((stats[r][k][..., 0] - stats[0][k][..., 0]).norm() / stats[0][k][..., 0].norm()) for r in range(1, 5))
    print(f"{k:26s} bwd Σg run spread {sp:.1e}")
# fp64 torch: cancellation ratio of each BN's output gradient
m = copy.deepcopy(model).double()
m.load_state_dict({k: v.double() if v.is_floating_point() else v for k, v in layout.unflatten(flat.cpu()).items()})
m.train()
grads = {}
for name, mod in m.named_modules():
    if isinstance(mod, torch.nn.BatchNorm2d):
        mod.register_full_backward_hook(lambda mod, gi, go, name=name: grads.__setitem__(name, go[0].detach()))
loss = torch.nn.functional.cross_entropy(m(x[0].cpu().double()), y[0].cpu())
loss.backward()
for name, g in grads.items():
    s = g.sum((0, 2, 3)).abs()
    a = g.abs().sum((0, 2, 3))
    print(f"{name:26s} Σ|g|/|Σg| median {float((a / s.clamp_min(1e-300)).median()):.1e} max {float((a / s.clamp_min(1e-300)).max()):.1e}")
