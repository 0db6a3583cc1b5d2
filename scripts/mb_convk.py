"""Microbenchmark of the wide-layer conv kernels on ResNet-18 shapes (C=10 clients, N=64 images):
forward / backward-data / weight-gradient time per call and TFLOP/s, next to MIOpen (torch conv2d
on one client × C, channels-last bf16) for the same GEMM.   python scripts/mb_convk.py [bf16|fp32]"""
import sys

import torch

from fedml_amd.ops import nn_ops

dt = torch.bfloat16 if (len(sys.argv) < 2 or sys.argv[1] == "bf16") else torch.float32
dev = "cuda"
C, N = 10, 64
SHAPES = [  # cin, cout, k, stride, hw(in)
    (64, 64, 3, 1, 32), (128, 128, 3, 1, 16), (256, 256, 3, 1, 8), (512, 512, 3, 1, 4), (256, 512, 3, 2, 8),
]


def timeit(fn, it=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3   # us


for cin, cout, k, stride, hw in SHAPES:
    pad = k // 2
    ho = (hw + 2 * pad - k) // stride + 1
    K, K2 = k * k * cin, k * k * cout
    ldk, ldk2 = (K + 31) // 32 * 32 + 8, (K2 + 31) // 32 * 32 + 8
    wf = (torch.randn(C, cout, ldk, device=dev) * 0.02).to(dt)
    wb = (torch.randn(C, cin, ldk2, device=dev) * 0.02).to(dt)
    x = torch.randn(C, N, hw, hw, cin, device=dev).to(dt)
    s = torch.rand(C, cin, device=dev) + 0.5
    t = torch.randn(C, cin, device=dev) * 0.1
    y = torch.zeros(C, N, ho, ho, cout, device=dev, dtype=dt)
    st = torch.zeros(C, cout, 2, device=dev)
    g = torch.randn_like(y)
    al, be, ga = torch.rand(C, cout, device=dev), torch.randn(C, cout, device=dev) * .1, torch.randn(C, cout, device=dev) * .01
    dx = torch.zeros_like(x)
    stb = torch.zeros(C, cin, 3, device=dev)
    P = cout * cin * k * k + 32
    garena = torch.zeros(C, P, device=dev)
    scratch = torch.zeros(C * cout * K, device=dev)
    flop = 2.0 * C * N * ho * ho * cout * K
    tf = timeit(lambda: nn_ops.conv_fwd(x, wf, cout * ldk, s, t, y, st, C, N, hw, hw, cin, cout, k, k, stride, pad, ho, ho,
                                        ldk, 1))
    tb = timeit(lambda: nn_ops.conv_bwd_data(g, y, al, be, ga, wb, cin * ldk2, dx, nn_ops.EPI_MASK, x, s, t, None, None,
                                             None, stb, C, N, ho, ho, cout, cin, k, k, stride, pad, hw, hw, ldk2, 1))
    tw = timeit(lambda: nn_ops.conv_wgrad(g, y, al, be, ga, x, s, t, garena, 16, C, N, hw, hw, cin, ho, ho, cout, k, k,
                                          stride, pad, 256, cin, scratch))
    xm = torch.randn(N, cin, hw, hw, device=dev, dtype=dt).to(memory_format=torch.channels_last)
    wm = torch.randn(cout, cin, k, k, device=dev, dtype=dt).to(memory_format=torch.channels_last)
    tm = timeit(lambda: [torch.nn.functional.conv2d(xm, wm, stride=stride, padding=pad) for _ in range(C)])
    print(f"{cin:4d}->{cout:4d} k{k} s{stride} hw{hw:3d}  GF {flop / 1e9:6.1f} | fwd {tf:7.1f}us {flop / tf / 1e6:6.1f}TF"
          f" | bwd {tb:7.1f}us {flop / tb / 1e6:6.1f}TF | wgrad {tw:7.1f}us {flop / tw / 1e6:6.1f}TF | miopen fwd "
          f"{tm:7.1f}us {flop / tm / 1e6:6.1f}TF", flush=True)
