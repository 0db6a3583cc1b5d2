"""Sweep pixels-per-workgroup for the fused 1×1 backward kernel at the ResNet-56 / C=100 shapes.

Prints one line per (shape, ppw): µs per call and the effective HBM rate of the minimal traffic
(g, y once; e_x once; out once; + e_add / e_y1 for the block epilogue)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fedml_amd.ops import nn_ops

SHAPES = [  # (cin, cout, epi, M per client)
    (16, 64, 2, 65536), (64, 16, 3, 65536), (32, 128, 2, 16384), (128, 32, 3, 16384), (64, 256, 2, 4096),
    (256, 64, 3, 4096), (16, 16, 3, 65536), (64, 32, 3, 65536), (128, 64, 3, 16384)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--C", type=int, default=100)
    ap.add_argument("--ppw", default="128,256,512,1024,2048")
    a = ap.parse_args()
    dev, bf, C = "cuda", torch.bfloat16, a.C
    for cin, cout, epi, M in SHAPES:
        g = torch.randn(C, M, cout, device=dev).to(bf)
        yv = torch.randn_like(g)
        al, be, ga = (torch.rand(C, cout, device=dev) for _ in range(3))
        ld = (cout + 31) // 32 * 32 + 8
        wb = (torch.randn(C, cin * ld, device=dev) * 0.05).to(bf)
        e_x = torch.randn(C, M, cin, device=dev).to(bf)
        s = t = e_add = e_y1 = None
        if epi == 2:
            s, t = torch.rand(C, cin, device=dev), torch.rand(C, cin, device=dev)
        else:
            e_add, e_y1 = torch.randn_like(e_x), torch.randn_like(e_x)
        out = torch.empty_like(e_x)
        stats = torch.zeros(C, cin, 3, device=dev)
        garena = torch.zeros(C, cin * cout + 16, device=dev)
        nbytes = C * M * (2 * cout + (2 if epi == 2 else 4) * cin) * 2
        for ppw, two in [(int(v), tp) for v in a.ppw.split(",") for tp in (False, True)]:
            part = torch.empty(nn_ops.conv1x1_bwd_fused_scratch(C, M, cin, cout, ppw), device=dev) if two else None

            def run():
                nn_ops.conv1x1_bwd_fused(g, yv, al, be, ga, wb, wb.stride(0), ld, e_x, s, t, e_add, e_y1, None, out,
                                         stats, garena, 0, C, M, cin, cout, epi, ppw, part)
            run()
            torch.cuda.synchronize()
            st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st.record()
            for _ in range(10):
                run()
            en.record()
            torch.cuda.synchronize()
            us = st.elapsed_time(en) * 100.0
            print(f"{cin:4d}<-{cout:<4d} epi{epi} M{M:<6d} ppw {ppw:5d} {'2pass' if two else 'atom '}: {us:8.1f} us"
                  f"  {nbytes / us / 1e3:7.0f} GB/s", flush=True)
            del part
        del g, yv, e_x, out, e_add, e_y1


if __name__ == "__main__":
    main()
