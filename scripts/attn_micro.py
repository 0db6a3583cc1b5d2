"""Attention forward / backward timing of the client-batched bf16 transformer kernels on the ViT-B/16 preset's shape
(32 clients x 16 images = 512 sequences, S 197, 12 heads of 64) — one JSON line; FEDML_AMD_ATTN_RP selects the
forward kernel.  python scripts/attn_micro.py [--S 197 --H 12 --CB 512 --iters 20]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--S", type=int, default=197)
    p.add_argument("--H", type=int, default=12)
    p.add_argument("--CB", type=int, default=512)
    p.add_argument("--iters", type=int, default=20)
    a = p.parse_args()
    import torch
    from fedml_amd.ops import transformer_ops as T
    dm = 64 * a.H
    qkv = torch.randn(a.CB * a.S, 3 * dm, device="cuda").to(torch.bfloat16).requires_grad_(True)
    q, k, v = qkv[:, :dm], qkv[:, dm:2 * dm], qkv[:, 2 * dm:]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    for _ in range(3):
        o = T.attention(q, k, v, a.S, a.H)
        o.backward(torch.ones_like(o))
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(a.iters):
        o = T.attention(q, k, v, a.S, a.H)
    ev[1].record()
    go = torch.randn_like(o)
    ev[2].record()
    for _ in range(a.iters):
        o = T.attention(q, k, v, a.S, a.H)
        o.backward(go)
    ev[3].record()
    torch.cuda.synchronize()
    fwd = ev[0].elapsed_time(ev[1]) / a.iters
    both = ev[2].elapsed_time(ev[3]) / a.iters
    flops = 4.0 * a.S * a.S * 64 * a.H * a.CB
    print(json.dumps({"metric": "attention ms", "S": a.S, "H": a.H, "CB": a.CB,
                      "rp": os.environ.get("FEDML_AMD_ATTN_RP", "1"), "fwd_ms": round(fwd, 3),
                      "fwd_TFs": round(flops / fwd / 1e9, 1), "fwd_bwd_ms": round(both, 3)}), flush=True)


if __name__ == "__main__":
    main()
