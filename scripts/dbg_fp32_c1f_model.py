#!/usr/bin/env python3
"""Same inputs through the native fp32 step with the fused 1×1 backward on and off: first BN (in
backward order) whose backward statistics differ, and per-slot gradient differences."""
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
res = []
for fused in ((os.environ.get("DBG_A", "0") == "1"), (os.environ.get("DBG_B", "1") == "1")):
    arena = flat.view(1, -1).repeat(C, 1).contiguous()
    garena = torch.zeros_like(arena)
    st = NativeResNetStep(model, layout, C, DEV, dtype=torch.float32)
    st.use_c1f = fused
    st.step(arena, garena, x, y, torch.full((C, N), 1.0 / N, device=DEV), torch.ones(C, device=DEV))
    torch.cuda.synchronize()
    res.append((garena.clone(), {k: (f.clone(), b.clone()) for k, (f, b) in st.stat_views.items()},
                {k: v.clone() for k, v in st.bn_vec.items()}))
(g0, s0, v0), (g1, s1, v1) = res
for k in s0:
    f0, b0 = s0[k]
    f1, b1 = s1[k]
    ef = float((f0 - f1).norm() / f0.norm().clamp_min(1e-30))
    eb = [float((b0[..., q] - b1[..., q]).norm() / b0[..., q].norm().clamp_min(1e-30)) for q in range(3)]
    ev = [float((v0[k][i] - v1[k][i]).norm() / v0[k][i].norm().clamp_min(1e-30)) for i in range(7)]
    print(f"{k:28s} fwd {ef:.1e} bwd " + " ".join(f"{e:.1e}" for e in eb) + " | vec " + " ".join(f"{e:.0e}" for e in ev))
for s in layout.slots:
    if s.trainable:
        sl = slice(s.offset, s.offset + s.numel)
        print(f"{s.key:32s} {float((g0[:, sl] - g1[:, sl]).norm() / g0[:, sl].norm()):.2e}")
# determinism of the raw forward activations and the backward g buffers
