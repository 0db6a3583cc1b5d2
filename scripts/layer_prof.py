#!/usr/bin/env python3
"""Per-kernel roofline table for one native ResNet training step (C clients × N samples).

Wraps every ``ops.nn_ops`` launch with HIP events, derives the ideal HBM bytes and MFMA flops of
each launch from its arguments, and prints time, achieved GB/s and TFLOP/s aggregated by
(op, geometry). Usage: python scripts/layer_prof.py [--C 100] [--N 64] [--model resnet56]
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from fedml_amd.core.arena import ParamLayout
from fedml_amd.models.cv.resnet import resnet18_cifar, resnet56, resnet110
from fedml_amd.ops import nn_ops
from fedml_amd.parallel.native_resnet import NativeResNetStep

REC = []
ES = [2]           # bytes per activation element (bf16 2, fp32 4)
ENABLED = [False]


def _wrap(name, cost):
    orig = getattr(nn_ops, name)

    def f(*a, **k):
        if not ENABLED[0]:
            return orig(*a, **k)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        r = orig(*a, **k)
        e.record()
        label, nbytes, flops = cost(*a)
        REC.append((name, label, s, e, nbytes, flops))
        return r
    setattr(nn_ops, name, f)


def c_fwd(x, wpk, ld, ps, pt, y, st, C, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, ldk, tpw):
    return (f"{KH}x{KW} {Cin}->{Cout} s{stride} @{H}" + (" +bnrelu" if ps is not None else ""),
            C * N * (H * W * Cin + Ho * Wo * Cout) * ES[0], 2 * C * N * Ho * Wo * Cout * KH * KW * Cin)


def c_pbout(yp, s, t, res, rs, rt, bout, wpk, ld, y, st, C, N, H, W, Cin, Cout, ldk, tpw, **kw):
    return (f"1x1 {Cin}->{Cout} @{H} +block-out", C * N * H * W * (3 * Cin + Cout) * ES[0], 2 * C * N * H * W * Cin * Cout)


def c_bwd(g, y, al, be, ga, wpk, ld, dx, epi, ex, es, et, eadd, ey1, ey2, st, C, N, Hy, Wy, Cout, Cin, KH, KW, stride,
          pad, Hx, Wx, ldk2, tpw):
    extra = {1: 0, 2: 1, 3: 3 + (ey2 is not None)}[epi]
    return (f"{KH}x{KW} {Cin}<-{Cout} s{stride} @{Hx} epi{epi}",
            C * N * (2 * Hy * Wy * Cout + (1 + extra) * Hx * Wx * Cin) * ES[0],
            2 * C * N * Hx * Wx * Cin * KH * KW * Cout)


def c_wgrad(g, y, al, be, ga, x, ps, pt, garena, woff, C, N, H, W, Cin, Ho, Wo, Cout, KH, KW, stride, pad, ppw, cs,
            scratch):
    return (f"{KH}x{KW} {Cin}->{Cout} s{stride} @{H}" + (" +bnrelu" if ps is not None else ""),
            C * N * (2 * Ho * Wo * Cout + H * W * Cin) * ES[0], 2 * C * N * Ho * Wo * Cout * KH * KW * Cin)


def c3_fwd(x, wpk, ld, ps, pt, y, st, C, N, H, W, Cin, Cout, ldk, stride=1):
    return c_fwd(x, wpk, ld, ps, pt, y, st, C, N, H, W, Cin, Cout, 3, 3, stride, 1, H // stride, W // stride, ldk, 0)


def c3_bwd(g, y, al, be, ga, wpk, ld, dx, ex, es, et, st, C, N, H, W, Cout, Cin, ldk2, stride=1):
    return c_bwd(g, y, al, be, ga, wpk, ld, dx, 2, ex, es, et, None, None, None, st, C, N, H // stride, W // stride,
                 Cout, Cin, 3, 3, stride, 1, H, W, ldk2, 0)


def c3_bwd_block(g, y, al, be, ga, wpk, ld, dx, ex, ea, e1, e2, st, C, N, H, W, Cout, Cin, ldk2):
    return c_bwd(g, y, al, be, ga, wpk, ld, dx, 3, ex, None, None, ea, e1, e2, st, C, N, H, W, Cout, Cin, 3, 3, 1, 1,
                 H, W, ldk2, 0)


def c3_wgrad(g, y, al, be, ga, x, ps, pt, garena, woff, C, N, H, W, Cin, Cout, cs, scratch, stride=1):
    return c_wgrad(g, y, al, be, ga, x, ps, pt, garena, woff, C, N, H, W, Cin, H // stride, W // stride, Cout, 3, 3,
                   stride, 1, 0, cs, scratch)


def c1_wgrad(g, y, al, be, ga, x, ps, pt, garena, woff, C, M, Cin, Cout, ppw):
    return (f"1x1 {Cin}->{Cout} M{M}" + (" +bnrelu" if ps is not None else ""), C * M * (2 * Cout + Cin) * ES[0],
            2 * C * M * Cout * Cin)


def c1_fused(g, y, al, be, ga, wpk, ld, ldk2, ex, es, et, eadd, ey1, ey2, out, st, garena, woff, C, M, Cin, Cout,
             epi, ppw):
    extra = 0 if epi == 2 else 2 + (ey2 is not None)
    return (f"1x1 {Cin}<-{Cout} M{M} epi{epi}", C * M * (2 * Cout + (2 + extra) * Cin) * ES[0], 4 * C * M * Cout * Cin)


def c_block(y, s, t, r, rs, rt, out, C, per, Ch):
    return (f"ch{Ch} n{per // Ch}" + (" ds" if rs is not None else ""), C * per * ES[0] * (3 if r is not None else 2), 0)


def c_other(*a):
    return ("", 0, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--C", type=int, default=100)
    ap.add_argument("--N", type=int, default=64)
    ap.add_argument("--model", default="resnet56")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--dtype", default="bf16", help="bf16 | fp32")
    ap.add_argument("--fp32-mma", default="exact", help="exact | bf16x3")
    a = ap.parse_args()
    dtype = {"bf16": torch.bfloat16, "fp32": torch.float32}[a.dtype]
    ES[0] = 2 if dtype == torch.bfloat16 else 4
    nn_ops.set_f32_mma_mode(a.fp32_mma)
    _wrap("conv_fwd", c_fwd)
    _wrap("conv_fwd_pbout", c_pbout)
    _wrap("conv_bwd_data", c_bwd)
    _wrap("conv_wgrad", c_wgrad)
    _wrap("block_out", c_block)
    _wrap("conv3x3_fwd", c3_fwd)
    _wrap("conv3x3_bwd_data", c3_bwd)
    _wrap("conv3x3_bwd_data_block", c3_bwd_block)
    _wrap("conv3x3_wgrad", c3_wgrad)
    _wrap("conv1x1_wgrad", c1_wgrad)
    _wrap("conv1x1_bwd_fused", c1_fused)
    for n in ("bn_fwd_finalize", "bn_bwd_finalize", "pack_weights", "avgpool", "head_bwd", "nchw_to_nhwc_pad"):
        _wrap(n, c_other)
    torch.manual_seed(0)
    model = {"resnet56": resnet56, "resnet110": resnet110, "resnet18": resnet18_cifar}[a.model](class_num=100)
    layout = ParamLayout.from_module(model)
    dev = "cuda"
    flat = layout.flatten(model.state_dict()).to(dev)
    arena = flat.view(1, -1).repeat(a.C, 1).contiguous()
    garena = torch.zeros_like(arena)
    x = torch.randn(a.C, a.N, 3, 32, 32, device=dev)
    y = torch.randint(0, 100, (a.C, a.N), device=dev)
    rs = torch.full((a.C, a.N), 1.0 / a.N, device=dev)
    act = torch.ones(a.C, device=dev)
    step = NativeResNetStep(model, layout, a.C, dev, dtype=dtype)
    for _ in range(2):
        step.step(arena, garena, x, y, rs, act)
    torch.cuda.synchronize()
    ENABLED[0] = True
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(a.steps):
        garena.zero_()
        step.step(arena, garena, x, y, rs, act)
    t1.record()
    torch.cuda.synchronize()
    ENABLED[0] = False
    total_ms = t0.elapsed_time(t1) / a.steps
    agg = collections.OrderedDict()
    for name, label, s, e, nb, fl in REC:
        k = (name, label)
        d = agg.setdefault(k, [0, 0.0, 0, 0])
        d[0] += 1
        d[1] += s.elapsed_time(e)
        d[2] += nb
        d[3] += fl
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    by_op = collections.Counter()
    print(f"step time {total_ms:.2f} ms  (C={a.C}, N={a.N}, {a.model}, {a.dtype}, fp32_mma {a.fp32_mma}); per-step")
    print(f"{'op':16s} {'geometry':34s} {'calls':>5s} {'ms':>8s} {'us/call':>8s} {'GB/s':>7s} {'TF/s':>6s}")
    for (name, label), (n, ms, nb, fl) in rows:
        ms_s = ms / a.steps
        by_op[name] += ms_s
        gbs = nb / (ms * 1e-3) / 1e9 if ms else 0
        tfs = fl / (ms * 1e-3) / 1e12 if ms else 0
        print(f"{name:16s} {label:34s} {n // a.steps:5d} {ms_s:8.3f} {1000 * ms / n:8.1f} {gbs:7.0f} {tfs:6.1f}")
    print("-- by op:", ", ".join(f"{k} {v:.2f} ms" for k, v in by_op.most_common()))
    print(f"-- kernels {sum(by_op.values()):.2f} ms of {total_ms:.2f} ms step (rest = torch head/zeroing/launch gaps)")
    # per-step budget: every kernel at the practical HBM ceiling or the matrix peak, whichever binds it
    hbm = float(os.environ.get("FEDML_AMD_HBM_TBS", "6.3")) * 1e12
    peak = (157.3e12 if a.fp32_mma == "exact" else 2.5e15 / 3) if a.dtype == "fp32" else 2.5e15
    nb_step = sum(v[2] for v in agg.values()) / a.steps
    fl_step = sum(v[3] for v in agg.values()) / a.steps
    bound_ms = sum(max(v[2] / hbm, v[3] / peak) * 1e3 for v in agg.values()) / a.steps
    print(f"-- budget: ideal {nb_step / 1e9:.2f} GB and {fl_step / 1e12:.3f} TFLOP per step; every kernel at "
          f"{hbm / 1e12:.1f} TB/s or {peak / 1e12:.0f} TF/s (whichever binds): {bound_ms:.2f} ms "
          f"= {100 * bound_ms / max(1e-9, sum(by_op.values())):.0f} % of the measured kernel time")


if __name__ == "__main__":
    main()
