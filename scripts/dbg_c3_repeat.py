#!/usr/bin/env python3
"""Repeated launches of the stride-2 3×3 backward-data kernel (model shape) on identical inputs:
bitwise spread of dx and relative spread of the statistics (fp32 and bf16)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedml_amd.ops import nn_ops  # noqa: E402

DEV = "cuda"
torch.manual_seed(0)
C, N, ch, hw, stride = 3, 16, 32, 16, 2
ho = hw // stride
K = 9 * ch
ldk = (K + 31) // 32 * 32 + 8
for dtype in (torch.float32,):
    wpk = torch.zeros(C, ch, ldk, device=DEV)
    wpk[:, :, :K] = torch.randn(C, ch, K, device=DEV) * 0.1
    wpk = wpk.to(dtype)
    s, t = torch.rand(C, ch, device=DEV) + 0.5, torch.randn(C, ch, device=DEV) * 0.1
    g = (torch.randn(C, N, ho, ho, ch, device=DEV) + 1.0).to(dtype)
    yv = torch.randn(C, N, ho, ho, ch, device=DEV).to(dtype)
    ex = torch.randn(C, N, hw, hw, ch, device=DEV).to(dtype)
    al, be, ga = torch.rand(C, ch, device=DEV), torch.randn(C, ch, device=DEV) * 0.1, torch.randn(C, ch, device=DEV)
    for kind in ("c3", "generic"):
        dxs, sts = [], []
        for r in range(40):
            dx = torch.empty(C, N, hw, hw, ch, device=DEV, dtype=dtype)
            st = torch.zeros(C, ch, 3, device=DEV)
            if kind == "c3":
                nn_ops.conv3x3_bwd_data(g, yv, al, be, ga, wpk, ch * ldk, dx, ex, s, t, st, C, N, hw, hw, ch, ch, ldk,
                                        stride)
            else:
                nn_ops.conv_bwd_data(g, yv, al, be, ga, wpk, ch * ldk, dx, nn_ops.EPI_MASK, ex, s, t, None, None, None,
                                     st, C, N, ho, ho, ch, ch, 3, 3, stride, 1, hw, hw, ldk, 1)
            dxs.append(dx)
            sts.append(st)
        torch.cuda.synchronize()
        neq = sum(0 if torch.equal(dxs[0], d) else 1 for d in dxs)
        sp0 = max(float((s_[..., 0] - sts[0][..., 0]).norm() / sts[0][..., 0].norm()) for s_ in sts)
        sp1 = max(float((s_[..., 1] - sts[0][..., 1]).norm() / sts[0][..., 1].norm()) for s_ in sts)
        ref0 = dxs[0].double().sum((1, 2, 3))
        e0 = float((sts[0][..., 0].double() - ref0).norm() / ref0.norm())
        print(f"{kind} {dtype}: dx differs in {neq}/40 runs; Σg spread {sp0:.1e} Σg·x spread {sp1:.1e}; "
              f"Σg vs fp64 sum of dx {e0:.1e}")
