"""Isolated timing of the fused FC + cross-entropy head (csrc/head_kernels.hip) at the ResNet-56 / CIFAR-100 shape:
C clients x N=64 rows, F=64 pooled features, K=100 classes.   python scripts/head_micro.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from fedml_amd.ops import nn_ops

dev = "cuda"
N, F, K = 64, 64, 100
for C in (13, 100):
    P = F * K + K + 16
    arena = torch.randn(C, P, device=dev) * 0.05
    garena = torch.zeros(C, P, device=dev)
    pooled = torch.randn(C, N, F, device=dev)
    labels = torch.randint(0, K, (C, N), device=dev)
    rs = torch.full((C, N), 1.0 / N, device=dev)
    dpool = torch.empty(C, N, F, device=dev)
    loss = torch.empty(C, device=dev)
    f = lambda: nn_ops.fc_head_xent(pooled, arena, 0, F * K, labels, rs, garena, dpool, loss, C, N, F, K)
    assert f()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(50):
        f()
    e.record()
    torch.cuda.synchronize()
    print(f"C={C}: {s.elapsed_time(e) / 50 * 1e3:.1f} us per head call", flush=True)
