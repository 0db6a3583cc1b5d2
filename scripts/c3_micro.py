"""Micro-driver for counter profiles of the LDS-tiled 3×3 kernels at the ResNet-56 / C=100 shapes
(each op launched --iters times on fixed random operands). Use under
``rocprofv3 --pmc ... --kernel-trace --stats -- python3 scripts/c3_micro.py``."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedml_amd.ops import nn_ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--C", type=int, default=100)
    ap.add_argument("--N", type=int, default=64)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--shapes", default="16x32,32x16,64x8")
    a = ap.parse_args()
    dev, bf, C, N = "cuda", torch.bfloat16, a.C, a.N
    for sh in a.shapes.split(","):
        ch, hw = (int(v) for v in sh.split("x"))
        K = 9 * ch
        ldk = (K + 31) // 32 * 32 + 8
        x = torch.randn(C, N, hw, hw, ch, device=dev).to(bf)
        g = torch.randn_like(x)
        yv = torch.randn_like(x)
        out = torch.empty_like(x)
        wpk = (torch.randn(C, ch * ldk, device=dev) * 0.05).to(bf)
        s, t = torch.rand(C, ch, device=dev) + 0.5, torch.randn(C, ch, device=dev) * 0.1
        al, be, ga = torch.rand(C, ch, device=dev), torch.randn(C, ch, device=dev) * 0.1, torch.zeros(C, ch, device=dev)
        st2 = torch.zeros(C, ch, 2, device=dev)
        st3 = torch.zeros(C, ch, 3, device=dev)
        garena = torch.zeros(C, ch * ch * 9 + 16, device=dev)
        scratch = torch.zeros(C * ch * ch * 9, device=dev)
        for _ in range(a.iters):
            nn_ops.conv3x3_fwd(x, wpk, wpk.stride(0), s, t, out, st2, C, N, hw, hw, ch, ch, ldk)
            nn_ops.conv3x3_bwd_data(g, yv, al, be, ga, wpk, wpk.stride(0), out, x, s, t, st3, C, N, hw, hw, ch, ch,
                                    ldk)
            nn_ops.conv3x3_wgrad(g, yv, al, be, ga, x, s, t, garena, 0, C, N, hw, hw, ch, ch, ch, scratch)
        torch.cuda.synchronize()
        print(f"{sh}: done", flush=True)


if __name__ == "__main__":
    main()
