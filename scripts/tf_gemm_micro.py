"""Micro-benchmark of the fp32 client-batched transformer GEMMs (tf_f32_kernels.hip) on the ViT-B/16 preset's
shapes: 32 clients × 16 images × 197 tokens, d 768, MLP 3072. Times forward / backward-data / backward-weight of
each linear with HIP events and prints achieved TF/s (fp32 matrix peak 157.3 TF/s).

    python scripts/tf_gemm_micro.py [--clients 32] [--rows 3152] [--iters 10]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=32)
    ap.add_argument("--rows", type=int, default=16 * 197)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--check", action="store_true", help="compare one output against torch.bmm (fp64)")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="bf16: bf16 activations and the arena's bf16 weight shadow (bgemm_kernels.hip)")
    a = ap.parse_args()
    from fedml_amd.ops import transformer_ops as T
    dev = torch.device("cuda:0")
    C, M = a.clients, a.rows
    shapes = {"qkv": (2304, 768), "proj": (768, 768), "fc1": (3072, 768), "fc2": (768, 3072)}
    g = torch.Generator(device=dev).manual_seed(0)
    out = []
    for name, (N, K) in shapes.items():
        bf = a.dtype == "bf16"
        x = torch.randn(C, M, K, device=dev, generator=g)
        x = (x.to(torch.bfloat16) if bf else x).requires_grad_(True)
        arena = torch.randn(C, N * K + N, device=dev, generator=g) * 0.02
        shadow = arena[:, :N * K].to(torch.bfloat16).view(C, N, K) if bf else None
        w = arena[:, :N * K].view(C, N, K).detach().requires_grad_(True)
        b = arena[:, N * K:].detach().requires_grad_(True)
        w.grad = torch.zeros_like(w)
        b.grad = torch.zeros_like(b)
        gelu = name == "fc1"
        gy = torch.randn(C, M, N, device=dev, generator=g).to(x.dtype)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        fl = 2.0 * C * M * N * K
        for it in range(a.iters + 2):
            if it == 2:
                torch.cuda.synchronize()
                ev[0].record()
            y = T.client_linear(x, [w], [b], gelu=gelu, shadows=[shadow] if bf else None)
            if it == 2:
                ev[1].record()
            y.backward(gy)
            if it == 2:
                ev[2].record()
            x.grad = None
        ev[3].record()
        torch.cuda.synchronize()
        fwd = ev[0].elapsed_time(ev[1])
        bwd = ev[1].elapsed_time(ev[2])
        tot = ev[0].elapsed_time(ev[3]) / a.iters
        rec = {"gemm": name, "dtype": a.dtype, "C": C, "M": M, "N": N, "K": K, "fwd_ms": round(fwd, 3), "fwd_TFs": round(fl / fwd / 1e9, 1),
               "bwd_ms": round(bwd, 3), "bwd_TFs": round(2 * fl / bwd / 1e9, 1),
               "iter_ms": round(tot, 3), "iter_TFs": round(3 * fl / tot / 1e9, 1)}
        if a.check:
            with torch.no_grad():
                ref = torch.bmm(x[:2].double(), w[:2].double().transpose(1, 2)) + b[:2].double().unsqueeze(1)
                if gelu:
                    ref = torch.nn.functional.gelu(ref)
                if bf:
                    ref = torch.bmm(x[:2].double(), shadow[:2].double().transpose(1, 2)) + b[:2].double().unsqueeze(1)
                    if gelu:
                        ref = torch.nn.functional.gelu(ref)
                yy = T.client_linear(x[:2].detach(), [w[:2].detach()], [b[:2].detach()], gelu=gelu,
                                     shadows=[shadow[:2]] if bf else None)
                rec["max_rel_err"] = float((yy.double() - ref).abs().max() / ref.abs().max())
        print(json.dumps(rec), flush=True)
        out.append(rec)
        del x, arena, w, b, gy, y
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
