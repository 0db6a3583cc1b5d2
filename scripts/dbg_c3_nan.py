#!/usr/bin/env python3
"""Output coverage: NaN-prefilled outputs of the 3×3 kernels must be fully overwritten."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedml_amd.ops import nn_ops  # noqa: E402

DEV = "cuda"
torch.manual_seed(0)
for dtype in (torch.float32, torch.bfloat16):
    for (C, N, ch, hw, stride) in [(3, 16, 32, 16, 2), (3, 16, 64, 16, 2), (3, 16, 16, 16, 1), (3, 16, 32, 32, 2),
                                   (100, 64, 32, 32, 2), (100, 64, 64, 16, 2), (3, 8, 32, 16, 2)]:
        ho = hw // stride
        K = 9 * ch
        ldk = (K + 31) // 32 * 32 + 8
        wpk = torch.zeros(C, ch, ldk, device=DEV)
        wpk[:, :, :K] = torch.randn(C, ch, K, device=DEV) * 0.1
        wpk = wpk.to(dtype)
        s, t = torch.rand(C, ch, device=DEV) + 0.5, torch.randn(C, ch, device=DEV) * 0.1
        g = torch.randn(C, N, ho, ho, ch, device=DEV).to(dtype)
        yv = torch.randn(C, N, ho, ho, ch, device=DEV).to(dtype)
        ex = torch.randn(C, N, hw, hw, ch, device=DEV).to(dtype)
        al, be, ga = torch.rand(C, ch, device=DEV), torch.randn(C, ch, device=DEV), torch.randn(C, ch, device=DEV)
        dx = torch.full((C, N, hw, hw, ch), float("nan"), device=DEV).to(dtype)
        st = torch.zeros(C, ch, 3, device=DEV)
        nn_ops.conv3x3_bwd_data(g, yv, al, be, ga, wpk, ch * ldk, dx, ex, s, t, st, C, N, hw, hw, ch, ch, ldk, stride)
        y3 = torch.full((C, N, ho, ho, ch), float("nan"), device=DEV).to(dtype)
        st3 = torch.zeros(C, ch, 2, device=DEV)
        nn_ops.conv3x3_fwd(ex, wpk, ch * ldk, s, t, y3, st3, C, N, hw, hw, ch, ch, ldk, stride)
        torch.cuda.synchronize()
        nb = torch.isnan(dx.float())
        nf = torch.isnan(y3.float())
        msg = ""
        if nb.any():
            idx = nb.nonzero()[:6].tolist()
            msg += f" bwd NaN count {int(nb.sum())} at [c,n,h,w,ch] {idx}"
        if nf.any():
            msg += f" fwd NaN count {int(nf.sum())} at {nf.nonzero()[:6].tolist()}"
        print(f"{dtype} C={C} N={N} ch={ch} hw={hw} s={stride}:{msg or ' ok'}")
