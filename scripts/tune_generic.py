#!/usr/bin/env python3
"""Sweep launch parameters of the generic conv kernels on the ResNet-56 layer shapes (C=100, N=64):
pix_per_wg for conv_wgrad, tiles_per_wave for conv_fwd / conv_bwd_data."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fedml_amd.ops import nn_ops

DEV, bf = "cuda", torch.bfloat16
C, N = 100, 64


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1000


shapes = [  # (Cin, Cout, H)  1x1 stride 1
    (16, 64, 32), (64, 16, 32), (32, 128, 16), (128, 32, 16), (64, 256, 8), (256, 64, 8)]
for cin, cout, H in shapes:
    M = N * H * H
    x = torch.randn(C, N, H, H, cin, device=DEV).to(bf)
    g = torch.randn(C, N, H, H, cout, device=DEV).to(bf)
    yv = torch.randn_like(g)
    al, be, ga = (torch.rand(C, cout, device=DEV) for _ in range(3))
    s, t = torch.rand(C, cin, device=DEV), torch.rand(C, cin, device=DEV)
    garena = torch.zeros(C, cout * cin + 64, device=DEV)
    scratch = torch.zeros(C * cout * cin, device=DEV)
    res = []
    for ppw in (128, 256, 512, 1024, 2048, 4096):
        us = timeit(lambda: nn_ops.conv_wgrad(g, yv, al, be, ga, x, s, t, garena, 16, C, N, H, H, cin, H, H, cout, 1,
                                              1, 1, 0, ppw, cin, scratch))
        res.append((round(us), ppw))
    print(f"wgrad 1x1 {cin}->{cout} @{H}: ", sorted(res)[:3], "all", res)
    # bwd data epi2 (mask) : dx [.., cin]
    ldk2 = (cout + 31) // 32 * 32 + 8
    wpk = torch.randn(C, cin * ldk2, device=DEV).to(bf)
    dx = torch.empty(C, N, H, H, cin, device=DEV, dtype=bf)
    ex = torch.randn_like(dx)
    st = torch.zeros(C, cin, 3, device=DEV)
    res = []
    for tpw in (1, 2, 4, 8, 16):
        us = timeit(lambda: nn_ops.conv_bwd_data(g, yv, al, be, ga, wpk, cin * ldk2, dx, nn_ops.EPI_MASK, ex, s, t,
                                                 None, None, None, st, C, N, H, H, cout, cin, 1, 1, 1, 0, H, H, ldk2,
                                                 tpw))
        res.append((round(us), tpw))
    print(f"bwd  1x1 {cin}<-{cout} @{H}: ", sorted(res)[:3], "all", res)
    ldk = (cin + 31) // 32 * 32 + 8
    wpf = torch.randn(C, cout * ldk, device=DEV).to(bf)
    y = torch.empty(C, N, H, H, cout, device=DEV, dtype=bf)
    st2 = torch.zeros(C, cout, 2, device=DEV)
    res = []
    for tpw in (1, 2, 4, 8, 16):
        us = timeit(lambda: nn_ops.conv_fwd(x, wpf, cout * ldk, s, t, y, st2, C, N, H, H, cin, cout, 1, 1, 1, 0, H, H,
                                            ldk, tpw))
        res.append((round(us), tpw))
    print(f"fwd  1x1 {cin}->{cout} @{H}: ", sorted(res)[:3], "all", res)
