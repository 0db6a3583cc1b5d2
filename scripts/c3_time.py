#!/usr/bin/env python3
"""Timing micro-benchmark of the LDS-tiled 3×3 kernels at the ResNet-56 / C=100 / N=64 shapes
(HIP-event timed, median of --iters), storage precision --dtype (fp32 | bf16). Prints TF/s per op."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedml_amd.ops import nn_ops  # noqa: E402


def timeit(fn, iters):
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--C", type=int, default=100)
    ap.add_argument("--N", type=int, default=64)
    ap.add_argument("--iters", type=int, default=7)
    ap.add_argument("--dtype", default="fp32")
    ap.add_argument("--shapes", default="16x32x1,32x16x1,64x8x1,32x32x2,64x16x2")
    a = ap.parse_args()
    dev, C, N = "cuda", a.C, a.N
    dt = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    tot = 0.0
    for sh in a.shapes.split(","):
        ch, hw, st = (int(v) for v in sh.split("x"))
        ho = hw // st
        K = 9 * ch
        ldk = (K + 31) // 32 * 32 + 8
        x = torch.randn(C, N, hw, hw, ch, device=dev).to(dt)
        g = torch.randn(C, N, ho, ho, ch, device=dev).to(dt)
        yv = torch.randn_like(g)
        out_f = torch.empty_like(g)
        out_b = torch.empty_like(x)
        wpk = (torch.randn(C, ch * ldk, device=dev) * 0.05).to(dt)
        s, t = torch.rand(C, ch, device=dev) + 0.5, torch.randn(C, ch, device=dev) * 0.1
        al, be, ga = torch.rand(C, ch, device=dev), torch.randn(C, ch, device=dev) * 0.1, torch.zeros(C, ch, device=dev)
        st2 = torch.zeros(C, ch, 2, device=dev)
        st3 = torch.zeros(C, ch, 3, device=dev)
        garena = torch.zeros(C, ch * ch * 9 + 16, device=dev)
        scratch = torch.zeros(C * ch * ch * 9, device=dev)
        flop = 2.0 * C * N * ho * ho * ch * ch * 9
        tf = timeit(lambda: nn_ops.conv3x3_fwd(x, wpk, wpk.stride(0), s, t, out_f, st2, C, N, hw, hw, ch, ch, ldk, st),
                    a.iters)
        tb = timeit(lambda: nn_ops.conv3x3_bwd_data(g, yv, al, be, ga, wpk, wpk.stride(0), out_b, x, s, t, st3, C, N,
                                                    hw, hw, ch, ch, ldk, st), a.iters)
        tw = timeit(lambda: nn_ops.conv3x3_wgrad(g, yv, al, be, ga, x, s, t, garena, 0, C, N, hw, hw, ch, ch, ch,
                                                 scratch, st), a.iters)
        tot += tf + tb + tw
        print(f"{sh:9s} fwd {tf:7.3f} ms {flop / tf / 1e9:6.1f} TF/s | bwd {tb:7.3f} ms {flop / tb / 1e9:6.1f} TF/s | "
              f"wgrad {tw:7.3f} ms {flop / tw / 1e9:6.1f} TF/s", flush=True)
    print(f"total {tot:.3f} ms")


if __name__ == "__main__":
    main()
