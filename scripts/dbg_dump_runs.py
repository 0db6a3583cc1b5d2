#!/usr/bin/env python3
"""Three fresh fp32 native steps on identical inputs: per backward gradient buffer, the relative
difference of runs 1 and 2 against run 0 (first buffer that diverges locates a race)."""
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
dumps = []
for r in range(6):
    arena = flat.view(1, -1).repeat(C, 1).contiguous()
    garena = torch.zeros_like(arena)
    st = NativeResNetStep(model, layout, C, DEV, dtype=torch.float32)
    st.dump = []
    st.step(arena, garena, x, y, torch.full((C, N), 1.0 / N, device=DEV), torch.ones(C, device=DEV))
    torch.cuda.synchronize()
    dumps.append(st.dump + [("stats", st.stats.clone()), ("garena", garena)])
for i, (name, t0) in enumerate(dumps[0]):
    diffs = []
    for r in range(1, len(dumps)):
        t = dumps[r][i][1]
        diffs.append(float((t - t0).norm() / t0.norm().clamp_min(1e-30)))
    nbad = [int(((dumps[r][i][1] - t0).abs() > 1e-3 * t0.abs().max()).sum()) for r in range(1, len(dumps))]
    print(f"{name:34s} " + " ".join(f"{d:.1e}" for d in diffs) + "  big-diff elems " + str(nbad))
