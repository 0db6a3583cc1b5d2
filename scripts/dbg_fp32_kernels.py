#!/usr/bin/env python3
"""fp32 kernel precision vs fp64: the fused 1×1 backward (c1f) against the generic data/weight-gradient
kernels on identical inputs (model shapes of ResNet(Bottleneck,[1,1,1]) at 16×16, N=16, C=3)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedml_amd.ops import nn_ops  # noqa: E402

DEV = "cuda"


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


torch.manual_seed(0)
C = 3
for cin, cout, epi, M, ppw in [(64, 32, 3, 4096, 256), (16, 64, 2, 4096, 256), (16, 16, 3, 4096, 256),
                               (32, 128, 2, 1024, 256), (128, 64, 3, 256, 256)]:
    g = torch.randn(C, M, cout, device=DEV)
    yv = torch.randn(C, M, cout, device=DEV) + 3.0
    al, be = torch.rand(C, cout, device=DEV), torch.randn(C, cout, device=DEV) * 0.1
    ga = torch.randn(C, cout, device=DEV) * 0.3
    W = torch.randn(C, cout, cin, device=DEV) / cin ** 0.5
    ld = (cout + 31) // 32 * 32 + 8
    wb = torch.zeros(C, cin * ld, device=DEV)
    wb.view(C, cin, ld)[:, :, :cout] = W.transpose(1, 2)
    e_x = torch.randn(C, M, cin, device=DEV)
    s = t = e_add = e_y1 = e_y2 = None
    if epi == 2:
        s, t = torch.rand(C, cin, device=DEV) + 0.5, torch.randn(C, cin, device=DEV) * 0.1
    else:
        e_add, e_y1, e_y2 = (torch.randn(C, M, cin, device=DEV) for _ in range(3))
    out = torch.empty(C, M, cin, device=DEV)
    stats = torch.zeros(C, cin, 3, device=DEV)
    garena = torch.zeros(C, cin * cout + 16, device=DEV)
    nn_ops.conv1x1_bwd_fused(g, yv, al, be, ga, wb, wb.stride(0), ld, e_x, s, t, e_add, e_y1, e_y2, out, stats,
                             garena, 16, C, M, cin, cout, epi, ppw)
    # generic kernels (same storage) for comparison
    hw = int(round((M / 16) ** 0.5)) if M >= 16 else 1
    N = M // (hw * hw)
    out2 = torch.empty_like(out)
    st2 = torch.zeros_like(stats)
    nn_ops.conv_bwd_data(g, yv, al, be, ga, wb, wb.stride(0), out2, epi, e_x, s, t, e_add, e_y1, e_y2, st2, C, N, hw,
                         hw, cout, cin, 1, 1, 1, 0, hw, hw, ld, 1)
    ga2 = torch.zeros_like(garena)
    scratch = torch.zeros(C * cout * cin, device=DEV)
    nn_ops.conv_wgrad(g, yv, al, be, ga, e_x, s, t, ga2, 16, C, N, hw, hw, cin, hw, hw, cout, 1, 1, 1, 0, 256, cin,
                      scratch)
    torch.cuda.synchronize()
    for c in range(1):
        d = lambda v: v[c].double()
        dy = d(al)[None] * d(g) + d(be)[None] * d(yv) + d(ga)[None]
        dx = dy @ d(W)
        xr = d(e_x)
        if epi == 2:
            gp = torch.where(xr * d(s) + d(t) > 0, dx, torch.zeros_like(dx))
            st = torch.stack([gp.sum(0), (gp * xr).sum(0)], -1)
            act = torch.relu(xr * d(s) + d(t))
        else:
            gp = torch.where(xr > 0, dx + d(e_add), torch.zeros_like(dx))
            st = torch.stack([gp.sum(0), (gp * d(e_y1)).sum(0), (gp * d(e_y2)).sum(0)], -1)
            act = xr
        dw = dy.t() @ act
        k = st.shape[-1]
        print(f"({cin},{cout},{epi}) M={M}: out c1f {rel(out[c], gp):.2e} gen {rel(out2[c], gp):.2e} | "
              f"stats c1f {rel(stats[c, :, :k], st):.2e} gen {rel(st2[c, :, :k], st):.2e} | "
              f"dW c1f {rel(garena[c, 16:].view(cout, cin), dw):.2e} gen {rel(ga2[c, 16:].view(cout, cin), dw):.2e}")
