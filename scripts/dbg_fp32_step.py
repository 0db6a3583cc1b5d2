#!/usr/bin/env python3
"""Per-slot gradient error of the fp32 native step vs an fp64 CPU reference (and torch fp32 GPU),
for localising precision loss to a kernel family (toggle FEDML_AMD_CONV3X3 / FEDML_AMD_C1_FUSED /
FEDML_AMD_CONV1X1 in the environment)."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedml_amd.core.arena import ParamLayout  # noqa: E402
from fedml_amd.models.cv.resnet import Bottleneck, ResNet  # noqa: E402
from fedml_amd.parallel.native_resnet import NativeResNetStep  # noqa: E402

DEV = "cuda"


def grads(model, layout, flat, x, y, dtype, device):
    C = x.shape[0]
    out = torch.zeros(C, layout.size, dtype=torch.float64)
    for c in range(C):
        m = copy.deepcopy(model).to(device=device, dtype=dtype)
        m.load_state_dict({k: v.to(device) for k, v in layout.unflatten(flat).items()})
        m.train()
        torch.nn.functional.cross_entropy(m(x[c].to(device=device, dtype=dtype)), y[c].to(device)).backward()
        sd = {k: p.grad for k, p in m.named_parameters()}
        for s in layout.slots:
            if s.key in sd:
                out[c, s.offset:s.offset + s.numel] = sd[s.key].reshape(-1).double().cpu()
    return out


torch.manual_seed(0)
model = ResNet(Bottleneck, [1, 1, 1], 10)
layout = ParamLayout.from_module(model)
C, N, hw = 3, 16, 16
flat = layout.flatten(model.state_dict()).to(DEV)
arena = flat.view(1, -1).repeat(C, 1).contiguous()
garena = torch.zeros_like(arena)
x = torch.randn(C, N, 3, hw, hw, device=DEV)
y = torch.randint(0, 10, (C, N), device=DEV)
step = NativeResNetStep(model, layout, C, DEV, dtype=torch.float32)
step.step(arena, garena, x, y, torch.full((C, N), 1.0 / N, device=DEV), torch.ones(C, device=DEV))
torch.cuda.synchronize()
g = garena.double().cpu()
print("nan in grads:", bool(torch.isnan(g).any()), "nan slots:",
      [s.key for s in layout.slots if s.trainable and torch.isnan(g[:, s.offset:s.offset + s.numel]).any()][:12])
r64 = grads(model, layout, flat.cpu().double(), x.cpu(), y.cpu(), torch.float64, "cpu")
r32 = grads(model, layout, flat, x, y, torch.float32, DEV)
for s in layout.slots:
    if not s.trainable:
        continue
    sl = slice(s.offset, s.offset + s.numel)
    r = r64[:, sl]
    e = float((g[:, sl] - r).norm() / r.norm())
    et = float((r32[:, sl] - r).norm() / r.norm())
    print(f"{s.key:32s} native {e:.2e}  torch32 {et:.2e}")
